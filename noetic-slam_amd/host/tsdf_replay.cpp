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
// usage: tsdf_replay <in.scans> <out.bricks> [voxel_size sdf_trunc [semantics]]
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
    if (argc >= 6 && std::string(argv[5]) == "voxblox") p.semantics = TSDF_SEM_VOXBLOX;
    File in(argv[1], "rb");
    if (!in.f) {
        std::perror(argv[1]);
        return 1;
    }
    tsdf_ctx* ctx = nullptr;
    int rc = tsdf_create(&p, &ctx);
    if (rc != TSDF_OK) return die(ctx, "tsdf_create", rc);

    // the callback body: one PointCloud2 per scan, integrated as it arrives (the library copies
    // the points before returning, so the buffer is reused at once)
    std::vector<uint8_t> cloud;
    uint64_t n_scans = 0;
    char magic[8] = {0};
    const bool topics = std::fread(magic, 1, 8, in.f) == 8 && std::memcmp(magic, "TSDFSTR2", 8) == 0;
    if (!topics) std::rewind(in.f);
    tsdf_map::MapCore core(ctx);
    for (; topics;) {  // the node's subscriptions, in arrival order
        char type = 0;
        int64_t t = 0;
        if (std::fread(&type, 1, 1, in.f) != 1) break;
        if (std::fread(&t, sizeof t, 1, in.f) != 1) break;
        if (type == 'P') {
            tsdf_map::Pose ps;
            ps.t_ns = t;
            if (std::fread(ps.p, sizeof(double), 3, in.f) != 3 ||
                std::fread(ps.q, sizeof(double), 4, in.f) != 4)
                break;
            rc = core.on_pose(ps);
        } else if (type == 'C') {
            uint64_t n = 0;
            uint32_t step = 0, xoff = 0;
            int32_t f64 = 0;
            if (std::fread(&n, sizeof n, 1, in.f) != 1 || std::fread(&step, 4, 1, in.f) != 1 ||
                std::fread(&xoff, 4, 1, in.f) != 1 || std::fread(&f64, 4, 1, in.f) != 1)
                break;
            cloud.resize((size_t)n * step);
            if (n && std::fread(cloud.data(), step, n, in.f) != n) break;
            rc = core.on_cloud(t, cloud.data(), n, step, xoff, f64);
        } else {
            std::fprintf(stderr, "tsdf_replay: bad record type %d\n", (int)type);
            tsdf_destroy(ctx);
            return 1;
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
    for (; !topics;) {
        uint64_t n = 0;
        uint32_t step = 0, xoff = 0;
        int32_t f64 = 0;
        double origin[3];
        if (std::fread(&n, sizeof n, 1, in.f) != 1) break;
        if (std::fread(&step, sizeof step, 1, in.f) != 1 ||
            std::fread(&xoff, sizeof xoff, 1, in.f) != 1 ||
            std::fread(&f64, sizeof f64, 1, in.f) != 1 ||
            std::fread(origin, sizeof(double), 3, in.f) != 3) {
            std::fprintf(stderr, "tsdf_replay: truncated header of scan %llu\n",
                         (unsigned long long)n_scans);
            tsdf_destroy(ctx);
            return 1;
        }
        cloud.resize((size_t)n * step);
        if (n && std::fread(cloud.data(), step, n, in.f) != n) {
            std::fprintf(stderr, "tsdf_replay: truncated data of scan %llu\n",
                         (unsigned long long)n_scans);
            tsdf_destroy(ctx);
            return 1;
        }
        rc = tsdf_integrate(ctx, cloud.data(), n, step, xoff, f64, origin);
        if (rc != TSDF_OK) {
            const int r = die(ctx, "tsdf_integrate", rc);
            tsdf_destroy(ctx);
            return r;
        }
        n_scans++;
    }

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
