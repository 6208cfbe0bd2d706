// tsdf_replay — a ROS-free C++ host driver of the C-ABI, shaped like tsdf_map_node's per-scan
// callback (the reference slot is Dliomapping_Node::callback_pcl_deskewed,
// src/dliomapping/dliomapping.cpp:64-81).  It links against ANY library exporting
// include/tsdf_hip.h — libtsdf_hip.so (MAP_BACKEND_IDX = 4) in production — so the node-side code
// path is exercised exactly as a C++ node would drive it.
//
// Input stream (little endian), one record per scan:
//     u64 n_points, u32 point_step, u32 xyz_offset, i32 xyz_is_f64, f64 origin[3],
//     n_points * point_step bytes (PointCloud2 data, e.g. dlio::Point records)
// terminated by end of file.  Or, a topic stream (the node's two subscriptions, interleaved in
// arrival order) starting with the 8 bytes "TSDFSTR2", then records:
//     'P' i64 stamp_ns, f64 position[3], f64 quaternion[4]            (robot/dlio/odom_node/pose)
//     'C' i64 stamp_ns, u64 n, u32 point_step, u32 xyz_offset, i32 xyz_is_f64, n * point_step bytes
//                                                   (robot/dlio/odom_node/pointcloud/deskewed)
// whose clouds are paired with the pose track at their stamps by tsdf_map::MapCore — the same
// object tsdf_map_node runs (host/tsdf_map_core.h).  Output: the map as exported by
// tsdf_export_bricks: u64 n_bricks, then n_bricks * (i32 coords[3]), n_bricks * 512 f32 sdf,
// n_bricks * 512 f32 w.
//
// usage: tsdf_replay <in.scans> <out.bricks> [voxel_size sdf_trunc [semantics [max_batch]]]
//   semantics: vdbfusion_f64 (the ABI default), vdbfusion (fp32), voxblox (1/z^2 weight, upstream's default) or
//   voxblox_const (use_const_weight); max_batch: scans per GPU batch (the node's ~max_batch).
// The time from the first integrate to the end of tsdf_sync is printed as the node-path rate.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tsdf_hip.h"
#include "tsdf_map_core.h"

namespace {

struct File {
    FILE* f;
    explicit File(const char* path, const char* mode) : f(std::fopen(path, mode)) {}
    ~File() {
        if (f) std::fclose(f);
    }
};

int die(tsdf_ctx* ctx, const char* what, int rc) {
    std::fprintf(stderr, "tsdf_replay: %s failed (%d): %s\n", what, rc,
                 ctx ? tsdf_last_error(ctx) : "");
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <in.scans> <out.bricks> [voxel sdf_trunc [voxblox]]\n",
                     argv[0]);
        return 2;
    }
    if (tsdf_abi_version() != TSDF_ABI_VERSION) {
        std::fprintf(stderr, "tsdf_replay: ABI %d, header %d\n", tsdf_abi_version(),
                     TSDF_ABI_VERSION);
        return 1;
    }
    tsdf_params p;
    tsdf_default_params(&p);
    if (argc >= 5) {
        p.voxel_size = std::atof(argv[3]);
        p.sdf_trunc = std::atof(argv[4]);
    }
    if (argc >= 6) {
        const std::string sem = argv[5];
        if (sem == "voxblox" || sem == "voxblox_const") p.semantics = TSDF_SEM_VOXBLOX;
        if (sem == "voxblox_const") p.depth_weight = 0;
        if (sem == "vdbfusion_f64") p.semantics = TSDF_SEM_VDBFUSION_F64;
        if (sem == "vdbfusion") p.semantics = TSDF_SEM_VDBFUSION;
    }
    if (argc >= 7) p.max_batch = (uint32_t)std::atoi(argv[6]);
    File in(argv[1], "rb");
    if (!in.f) {
        std::perror(argv[1]);
        return 1;
    }
    tsdf_ctx* ctx = nullptr;
    int rc = tsdf_create(&p, &ctx);
    if (rc != TSDF_OK) return die(ctx, "tsdf_create", rc);

    // The input is read into memory first (one buffer per message, owned like a ROS ConstPtr), so
    // the timed part is the node's work: the callback bodies, the library's staging and the GPU.
    struct Msg {
        char type;
        int64_t t;
        tsdf_map::Pose pose;
        uint64_t n;
        uint32_t step, xoff;
        int32_t f64;
        double origin[3];
        std::shared_ptr<std::vector<uint8_t>> data;
    };
    std::vector<Msg> msgs;
    char magic[8] = {0};
    const bool topics = std::fread(magic, 1, 8, in.f) == 8 && std::memcmp(magic, "TSDFSTR2", 8) == 0;
    if (!topics) std::rewind(in.f);
    for (;;) {
        Msg m{};
        if (topics) {
            if (std::fread(&m.type, 1, 1, in.f) != 1) break;
            if (std::fread(&m.t, sizeof m.t, 1, in.f) != 1) break;
            if (m.type == 'P') {
                m.pose.t_ns = m.t;
                if (std::fread(m.pose.p, sizeof(double), 3, in.f) != 3 ||
                    std::fread(m.pose.q, sizeof(double), 4, in.f) != 4)
                    break;
                msgs.push_back(m);
                continue;
            }
            if (m.type != 'C') {
                std::fprintf(stderr, "tsdf_replay: bad record type %d\n", (int)m.type);
                tsdf_destroy(ctx);
                return 1;
            }
        } else {
            m.type = 'S';
        }
        if (std::fread(&m.n, sizeof m.n, 1, in.f) != 1) break;
        if (std::fread(&m.step, 4, 1, in.f) != 1 || std::fread(&m.xoff, 4, 1, in.f) != 1 ||
            std::fread(&m.f64, 4, 1, in.f) != 1 ||
            (!topics && std::fread(m.origin, sizeof(double), 3, in.f) != 3)) {
            std::fprintf(stderr, "tsdf_replay: truncated record %zu\n", msgs.size());
            tsdf_destroy(ctx);
            return 1;
        }
        m.data = std::make_shared<std::vector<uint8_t>>((size_t)m.n * m.step);
        if (m.n && std::fread(m.data->data(), m.step, m.n, in.f) != m.n) {
            std::fprintf(stderr, "tsdf_replay: truncated data of record %zu\n", msgs.size());
            tsdf_destroy(ctx);
            return 1;
        }
        msgs.push_back(std::move(m));
    }

    // the callback bodies: scans go through MapCore (topic stream: the node's object) or straight
    // to tsdf_integrate (one PointCloud2 per scan; the library copies the points before it returns)
    uint64_t n_scans = 0;
    tsdf_map::MapCore core(ctx);
    // the rate is timed after the first WARM scans (kernel loading, the pool's first bricks)
    const uint64_t WARM = 32;
    auto t_start = std::chrono::steady_clock::now();
    uint64_t scans_at_start = 0;
    bool warm = false;
    for (Msg& m : msgs) {
        const uint64_t done = topics ? core.counts().integrated : n_scans;
        if (!warm && done >= WARM) {
            rc = tsdf_sync(ctx);
            if (rc != TSDF_OK) return die(ctx, "tsdf_sync", rc);
            t_start = std::chrono::steady_clock::now();
            scans_at_start = done;
            warm = true;
        }
        if (m.type == 'P') {
            rc = core.on_pose(m.pose);
        } else if (m.type == 'C') {
            // MapCore shares the message (released after the timed part: freeing a 4 MB buffer
            // is an munmap, which a ROS node pays after its callback, not inside it)
            rc = core.on_cloud(m.t, m.data, m.data->data(), m.n, m.step, m.xoff, m.f64);
        } else {
            rc = tsdf_integrate(ctx, m.data->data(), m.n, m.step, m.xoff, m.f64, m.origin);
            n_scans++;
        }
        if (rc != TSDF_OK) {
            const int r = die(ctx, "tsdf_integrate", rc);
            tsdf_destroy(ctx);
            return r;
        }
    }
    if (topics) {
        rc = core.flush();
        if (rc != TSDF_OK) return die(ctx, "tsdf_integrate", rc);
        n_scans = core.counts().integrated;
        std::printf("tsdf_replay: paired %llu clouds, dropped %llu (outside the track) %llu (gap) "
                    "%llu (queue)\n", (unsigned long long)core.counts().integrated,
                    (unsigned long long)core.counts().dropped_old,
                    (unsigned long long)core.counts().dropped_gap,
                    (unsigned long long)core.counts().dropped_queue);
    }
    rc = tsdf_sync(ctx);
    if (rc != TSDF_OK) return die(ctx, "tsdf_sync", rc);
    const double secs =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    const uint64_t timed = n_scans - scans_at_start;
    std::printf("tsdf_replay: rate %.1f scans/s (%llu scans after %llu warm-up in %.3f s, "
                "callbacks + integrate + sync)\n",
                secs > 0 ? (double)timed / secs : 0.0, (unsigned long long)timed,
                (unsigned long long)scans_at_start, secs);

    // the node's map write-out
    uint64_t nb = 0;
    rc = tsdf_num_bricks(ctx, &nb);
    if (rc != TSDF_OK) return die(ctx, "tsdf_num_bricks", rc);
    std::vector<int32_t> coords(3 * nb);
    std::vector<float> sdf(512 * nb), w(512 * nb);
    uint64_t got = 0;
    rc = tsdf_export_bricks(ctx, coords.data(), sdf.data(), w.data(), nb, &got);
    if (rc != TSDF_OK) return die(ctx, "tsdf_export_bricks", rc);
    tsdf_stats st;
    tsdf_get_stats(ctx, &st);
    tsdf_destroy(ctx);
    File out(argv[2], "wb");
    if (!out.f) {
        std::perror(argv[2]);
        return 1;
    }
    std::fwrite(&got, sizeof got, 1, out.f);
    std::fwrite(coords.data(), sizeof(int32_t), 3 * got, out.f);
    std::fwrite(sdf.data(), sizeof(float), 512 * got, out.f);
    std::fwrite(w.data(), sizeof(float), 512 * got, out.f);
    std::printf("tsdf_replay: %llu scans, %llu points, %llu bricks\n",
                (unsigned long long)n_scans, (unsigned long long)st.n_points_in,
                (unsigned long long)got);
    return 0;
}
