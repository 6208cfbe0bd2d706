/*
 * tsdf_hip.h — C-ABI of the MI355X-native TSDF integration backend (MAP_BACKEND_IDX = 4).
 *
 * The reference has no runtime plugin API for this path: backends are chosen by a compile-time
 * switch `MAP_BACKEND_IDX` in the (unshipped) tsdf_map_node (reference README.md:44-50), and the
 * node's per-scan slot is the subscriber callback that today lives in
 * src/dliomapping/dliomapping.cpp:64-81 (`callback_pcl_deskewed`, fed by
 * `robot/dlio/odom_node/pointcloud/deskewed`, dliomapping.cpp:44).  The backend semantics this
 * ABI implements are VDBFusion's `VDBVolume::Integrate(points, origin, weighting_function)`
 * (backend idx 3, named in README.md:48,75; not vendored — restated in DESIGN.md §2).
 *
 * Every entry point below replaces one operation that node performs on its backend:
 *   tsdf_create            <- backend construction (VDBVolume(voxel_size, sdf_trunc, space_carving))
 *   tsdf_integrate         <- backend.Integrate(cloud, origin) inside callback_pcl_deskewed
 *                             (dliomapping.cpp:64-81; cloud layout dlio::Point, dlio.h:85-106)
 *   tsdf_integrate_device  <- same, input already resident in HBM (bench / batched replay)
 *   tsdf_integrate_batch_device <- a sequence of Integrate calls, one per scan, in order
 *   tsdf_query_dense / tsdf_export_bricks <- the node's map write-out (dliomapping.cpp:53-61,72-80
 *                             write PLY; .gitignore:9-15 hints the TSDF node wrote .grid/.h5)
 *   tsdf_import_bricks     <- resume from an exported map (checkpoint) / multi-GPU border merge
 *   tsdf_destroy           <- node destructor (dliomapping.cpp:53-61)
 *
 * Conventions: plain C types only; no exceptions cross the ABI; every call returns a status
 * (TSDF_OK = 0, negative on error; tsdf_last_error() has the message).  One context is used by one
 * host thread at a time (the ROS callback thread).  A context owns one HIP device, one stream, the
 * brick hash table and the brick pool.  Host-pointer integrate copies the caller's points into
 * pinned staging before returning; the GPU work itself is stream-ordered and may still be running
 * when the call returns — tsdf_sync() / query / export block.
 */
#ifndef TSDF_HIP_H
#define TSDF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSDF_ABI_VERSION 10
#define TSDF_MAX_BATCH 512 /* scans per GPU batch (see tsdf_params.max_batch) */
#define TSDF_BRICK_SIDE 8 /* voxels per brick edge: a brick is 8^3 = 512 voxels */

/* status codes */
#define TSDF_OK 0
#define TSDF_EINVAL (-1)    /* bad argument */
#define TSDF_ENOMEM (-2)    /* host/device allocation failed, or brick pool / hash / pair buffer full */
#define TSDF_EHIP (-3)      /* HIP runtime error (message in tsdf_last_error) */
#define TSDF_ENODEV (-4)    /* no usable GPU */
#define TSDF_EOVERFLOW (-5) /* caller buffer too small */

/* weighting functions (VDBFusion's weighting_function argument; default constant 1) */
#define TSDF_WEIGHT_CONSTANT 0

/* Backend semantics (tsdf_params.semantics).  The node's MAP_BACKEND_IDX chooses between CPU
 * backends with different fusion rules (reference README.md:44-50); this backend restates two:
 *   TSDF_SEM_VDBFUSION  backend idx 3, VDBVolume::Integrate
 *   TSDF_SEM_VOXBLOX    backend idx 2, voxblox SimpleTsdfIntegrator with use_const_weight
 *                       (DESIGN.md §2b): projective sdf, behind-surface weight
 *                       dropoff, clearing rays, fused distance clamped to +-tau, weight capped at
 *                       max_weight, background (distance 0, weight 0). */
#define TSDF_SEM_VDBFUSION 0
#define TSDF_SEM_VOXBLOX 1
/* VDBFusion at upstream's own precisions: the Ray<float> built from double points
 * and mapped to index space through the grid transform, openvdb's float DDA, GetVoxelCenter /
 * ComputeSDF in double.  Same touched voxels and weights as VDBVolume::Integrate; the GPU's fp64
 * sample arithmetic makes it slower than TSDF_SEM_VDBFUSION (the fp32 restatement). */
#define TSDF_SEM_VDBFUSION_F64 2

typedef struct tsdf_params {
    double voxel_size;     /* metres (VDBVolume voxel_size) */
    double sdf_trunc;      /* metres, truncation tau (VDBVolume sdf_trunc) */
    int32_t space_carving; /* 0: band [d-tau, d+tau]; 1: [0, d+tau] (VDBVolume space_carving) */
    int32_t weight_mode;   /* TSDF_WEIGHT_CONSTANT */
    double min_range;      /* rays with depth < min_range are dropped (Ouster r=0 -> (0,0,0)) */
    double max_range;      /* rays with depth > max_range are dropped */
    uint64_t max_bricks;   /* brick pool capacity (each brick: 512 x (sdf f32, weight f32) = 4 KiB) */
    uint64_t max_points;   /* per-scan point capacity */
    uint64_t max_pairs;    /* cap on (ray, brick) pair slots per batch; 0 = derive */
    int32_t device_id;     /* HIP device ordinal */
    int32_t brick_side;    /* must be TSDF_BRICK_SIDE */
    uint32_t max_batch;    /* scans integrated per GPU batch, 1..TSDF_MAX_BATCH (default 32) */
    uint32_t pipeline;     /* 1: overlap consecutive batches on two streams (count / compact /
                              place of batch b+1 run beside batch b's place / integrate; same field,
                              bit for bit); 2: only count / compact of batch b+1 beside batch b's
                              integrate, place always alone; 0 (default): batches run one after
                              another, so per-kernel timings (tsdf_stats.kernel_ms) are not shared
                              with another batch */
    /* ABI v3: backend semantics */
    int32_t semantics;          /* TSDF_SEM_VDBFUSION_F64 (default since ABI v8: the mode that
                                   matches VDBFusion's touched voxels and weights exactly),
                                   TSDF_SEM_VDBFUSION (fp32 restatement) or TSDF_SEM_VOXBLOX */
    int32_t allow_clear;        /* Voxblox allow_clear: a ray longer than max_range becomes a
                                   clearing ray of length min(max(d - tau, 0), max_range) (default 1) */
    int32_t use_weight_dropoff; /* Voxblox use_weight_dropoff: w *= (tau + sdf) / (tau - voxel_size)
                                   for sdf < -voxel_size, floored at 0 (default 1) */
    float max_weight;           /* Voxblox max_weight: the fused weight is capped here (default 1e4) */
    /* ABI v4: azimuth-sector sharding (multi-GPU, one context per GPU).  With
     * n_sectors > 1 a context integrates only the rays whose azimuth around their scan's origin
     * lies in sector `sector` of n_sectors equal sectors starting at sector_yaw0 (world frame);
     * the other rays are dropped like out-of-range ones, inside the walk kernels.  The rule is
     * tsdf_sector_of's: every ray belongs to exactly one sector. */
    uint32_t n_sectors;  /* 0 or 1: no sharding (default) */
    uint32_t sector;     /* 0 .. n_sectors - 1 */
    double sector_yaw0;  /* radians */
    /* ABI v4: capacity growth.  max_bricks is the INITIAL pool; when a batch overflows the brick
     * pool / hash table / work lists, the context grows them (x2 or more, up to max_bricks_hard
     * bricks and device memory) and re-runs the batches from the failed one, so no update is lost
     * (DESIGN.md §4b).  0 = no limit but device memory; max_bricks_hard == max_bricks = fixed
     * capacity: an overflow then drops the updates that do not fit and tsdf_sync reports
     * TSDF_ENOMEM. */
    uint64_t max_bricks_hard;
    /* ABI v5: front end of the batch pipeline.  TSDF_WALK_TWO (default): every ray
     * is walked twice (k_count counts, k_place writes each brick's samples contiguously).
     * TSDF_WALK_SINGLE: every ray is walked ONCE (k_walk keeps its samples in registers, stages
     * them per workgroup and writes them linearly; k_spans lists each brick's samples as spans)
     * whenever the band's walk has a proven bound of at most 32 voxels and 4 bricks per ray (no
     * space carving, no Voxblox clearing rays), else twice.  The field is bit for bit the same
     * either way; the single walk measures slower on MI355X. */
    int32_t walk;
    /* ABI v6: Voxblox's sample weight (TSDF_SEM_VOXBLOX only).  1 (tsdf_default_params; voxblox
     * TsdfIntegratorBase::Config use_const_weight = false, upstream's default): w = 1 / z^2, z the
     * point's depth along the sensor's z axis (|z| <= 1e-6: w = 0), the axis taken from the scan's
     * pose (tsdf_integrate_pose and the *_pose batch calls); then the dropoff.  Since ABI v8 the
     * per-sample weight is capped at min(max_weight, TSDF_W0_CAP) (without a cap a point near the
     * sensor plane, |z| ~ 1e-5, overflows the exact fixed-point sums), and scans given as a bare
     * origin (tsdf_integrate, tsdf_integrate_device, tsdf_integrate_batch_device) carry no
     * orientation and take w = 1.  0: w = 1 (use_const_weight = true). */
    int32_t depth_weight;
    /* ABI v8: Voxblox's integrator (TSDF_SEM_VOXBLOX only; voxblox_ros TsdfServer `method`).
     * TSDF_VB_SIMPLE (default): every point casts its own ray (SimpleTsdfIntegrator).
     * TSDF_VB_MERGED: MergedTsdfIntegrator -- a scan's points are bundled by the voxel they fall in
     * (getGridIndexFromPoint), each bundle's weighted mean point casts ONE ray carrying the summed
     * point weights, and clearing points are bundled apart (one ray from each bundle's first
     * point).  Bundles are formed in cloud order (voxblox integration_order_mode "sorted";
     * DESIGN.md §2d states the deviations).  "fast" (FastTsdfIntegrator) is not offered: its ray
     * early-exit depends on thread timing, so its field is not reproducible. */
    int32_t voxblox_method;
    /* ABI v8: how tsdf_integrate_sectors hands a host cloud to its n sector contexts.
     * TSDF_SECTOR_INPUT_FANOUT (default): packed once, one H2D copy to the first context's GPU,
     * then device-to-device (xGMI peer) copies to the others; every context's kernels drop the
     * other sectors' rays.  TSDF_SECTOR_INPUT_H2D: packed once, each context copies the packed
     * cloud over its own PCIe link.  TSDF_SECTOR_INPUT_SPLIT: classified and split on the host,
     * each context receives only its sector's points (round 3's path).  Read from ctxs[0]. */
    int32_t sector_input;
    /* ABI v10: which rays are sector k's (n_sectors > 1).
     * TSDF_SECTOR_RULE_INDEX (default): each cloud's points are split into n_sectors
     * contiguous index ranges, sector k holding points [floor(k n / N), floor((k + 1) n / N)) of
     * an n-point cloud.  DLIO's deskewed cloud is sorted by point time (reference
     * src/dlio/src/dlio/odom.cc:635-636) and an Ouster column is one firing time
     * (src/ouster/src/os_ros.cpp:195-229), so these are contiguous column (azimuth) ranges of the
     * spin in the sensor frame.  A context then reads, receives and walks only its share of every
     * cloud: the host entry points copy only the share, the device batch entry points read only
     * it, and no kernel classifies points.
     * TSDF_SECTOR_RULE_WORLD: the world-frame pseudo-angle sectors of tsdf_sector_of (ABI v4-v9's
     * only rule): a brick's owner stays fixed while the sensor turns, at the price of every
     * context reading every point (the kernels drop the other sectors' rays).
     * Either rule partitions each cloud's rays, so the reduced field is the unsharded one. */
    int32_t sector_rule;
} tsdf_params;

#define TSDF_SECTOR_RULE_WORLD 0
#define TSDF_SECTOR_RULE_INDEX 1

#define TSDF_VB_SIMPLE 0
#define TSDF_VB_MERGED 1
#define TSDF_SECTOR_INPUT_FANOUT 0
#define TSDF_SECTOR_INPUT_H2D 1
#define TSDF_SECTOR_INPUT_SPLIT 2

/* cap of one sample's 1/z^2 weight (with max_weight, whichever is lower; ABI v8) */
#define TSDF_W0_CAP 65536.0f

#define TSDF_WALK_TWO 0
#define TSDF_WALK_SINGLE 1

/* Batching.  Scans are integrated in call order and the field after any sequence of calls is
 * bitwise the one scan-at-a-time integration gives; the GPU merely processes up to max_batch
 * consecutive scans per launch sequence (rays of all of them walk together; each brick applies
 * its per-scan fuses in scan order).  Host-pointer scans (tsdf_integrate) and single device scans
 * (tsdf_integrate_device) are copied to device staging at once and queued until max_batch are
 * pending; any other call (sync, query, export, import, stats, tsdf_integrate_batch_device)
 * flushes the queue first. */

typedef struct tsdf_stats {
    uint64_t n_scans;          /* scans integrated (queued scans are flushed first) */
    uint64_t n_points_in;      /* points handed in */
    uint64_t n_bricks;         /* allocated bricks */
    uint64_t n_pairs_last;     /* (ray, brick) pairs of the last batch */
    uint64_t n_active_last;    /* bricks touched by the last batch */
    uint64_t n_voxels_last;    /* sum over the last batch's scans of their unique voxels */
    uint64_t n_voxels_total;   /* sum over scans of U_vox (unique voxels of the scan) since reset */
    uint64_t n_rays_total;     /* valid rays (after the range filter) since reset */
    uint64_t n_dirty_total;    /* sum over batches of the distinct voxels the batch updated */
    uint64_t n_batches;        /* GPU batches launched since reset */
    double kernel_ms[8];       /* per-kernel-kind accumulated device time when profiling is on */
    uint64_t kernel_launches[8];
    /* ABI v4 */
    uint64_t n_grows;          /* capacity growths since create */
    uint64_t n_replayed;       /* batches re-run after a growth since create */
    uint64_t max_bricks;       /* current brick pool capacity */
    /* ABI v8 */
    uint64_t peer_mask;        /* contexts of tsdf_create_sharded: bit j set when context j's
                                  device memory is directly reachable from this context's device
                                  (the same device, or peer access enabled: xGMI); 0 otherwise */
} tsdf_stats;

/* kernel kinds reported in tsdf_stats.kernel_ms (profiling on) */
#define TSDF_K_COUNT 0     /* k_count: ray walk, per-workgroup LDS brick hash, (ray, brick) pairs */
#define TSDF_K_COMPACT 1   /* k_compact: per-brick sample segments, pool slots, per-scan prefix */
#define TSDF_K_PLACE 2     /* k_place: second walk, samples staged in LDS, written per brick run */
#define TSDF_K_INTEGRATE 3 /* k_integrate: per-brick live-cell accumulate + scan-ordered fuse */
#define TSDF_K_WALK 4      /* k_walk: the single walk (samples staged per workgroup, linear write) */
#define TSDF_K_SPANS 5     /* k_spans: per-brick span lists of the single walk's samples */

typedef struct tsdf_ctx tsdf_ctx;

/* Fill *p with the defaults (5 cm voxel, 15 cm trunc, no carving, 1M bricks, 262144 points). */
void tsdf_default_params(tsdf_params* p);
int tsdf_abi_version(void);

int tsdf_create(const tsdf_params* params, tsdf_ctx** out);
void tsdf_destroy(tsdf_ctx* ctx);
const char* tsdf_last_error(const tsdf_ctx* ctx);

/* One scan from host memory, in any PointCloud2-like layout: point i's x,y,z are at
 * (const char*)pts + i*point_step + xyz_offset, as three consecutive float32 (xyz_is_f64 = 0,
 * e.g. dlio::Point: point_step 32, xyz_offset 0) or float64 (xyz_is_f64 = 1).  origin is the
 * sensor position in the same (world) frame.  The points are copied before the call returns;
 * the scan joins the pending batch (see Batching). */
int tsdf_integrate(tsdf_ctx* ctx, const void* pts, uint64_t n, uint32_t point_step,
                   uint32_t xyz_offset, int32_t xyz_is_f64, const double origin[3]);

/* ABI v9: tsdf_integrate_sectors with a bare origin instead of a pose: like tsdf_integrate, the
 * scan carries no orientation, so Voxblox takes the constant weight (a bare origin on the
 * sectors path was given an identity orientation, i.e. world-z 1/z^2 weights, so the sharded field
 * differed from the unsharded tsdf_integrate one). */
int tsdf_integrate_sectors_origin(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts,
                                  uint64_t n, uint32_t point_step, uint32_t xyz_offset,
                                  int32_t xyz_is_f64, const double origin[3]);

/* ABI v6: tsdf_integrate with the sensor's full pose: pose = (x, y, z, qx, qy, qz, qw), the
 * position (the ray origin) and orientation of the sensor in the world frame, in
 * geometry_msgs/Pose order (DLIO's /robot/dlio/odom_node/pose, odom.cc:315-356).  The orientation
 * gives the sensor z axis of Voxblox's 1/z^2 weight (tsdf_params.depth_weight); VDBFusion ignores
 * it.  The quaternion need not be normalised. */
int tsdf_integrate_pose(tsdf_ctx* ctx, const void* pts, uint64_t n, uint32_t point_step,
                        uint32_t xyz_offset, int32_t xyz_is_f64, const double pose[7]);

/* ABI v6: the live multi-GPU input path.  One host cloud for n_ctx contexts that
 * shard it by azimuth sector, one context per GPU: ctxs[k] was created with n_sectors = n_ctx,
 * sector = k and the same sector_yaw0 (n_ctx = 1: one unsharded context).  ABI v8:
 * ctxs[0]'s tsdf_params.sector_input picks the transfer: by default the cloud is packed once,
 * crosses PCIe once to the first context's GPU and is copied device to device (xGMI) to the
 * others, whose kernels drop the other sectors' rays; TSDF_SECTOR_INPUT_SPLIT classifies every
 * point on the host (tsdf_sector_of's rule) and each context receives only its sector's points.
 * The fields are the same bit for bit.  pose as in tsdf_integrate_pose.  Call from the one thread
 * that uses these contexts; each context's queue behaves as after tsdf_integrate_pose. */
int tsdf_integrate_sectors(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts, uint64_t n,
                           uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64,
                           const double pose[7]);

/* One scan already in device memory: d_xyz = n packed float32 triplets (12 B per point).  The
 * points are copied (device to device) into the pending batch's staging before the call returns,
 * so d_xyz may be reused or freed at once; the scan joins the pending batch like a host scan (see
 * Batching).  (ABI v6; before, the scan launched at once and d_xyz had to stay valid until the next
 * tsdf_sync.)  The call blocks until that copy has run: when the scan opens a new pending batch,
 * that includes waiting for the batch launched two batches earlier, the last reader of the
 * staging buffer the copy overwrites.  Batches of device scans that need not block use
 * tsdf_integrate_batch_device. */
int tsdf_integrate_device(tsdf_ctx* ctx, const float* d_xyz, uint64_t n, const double origin[3]);

/* n_scans scans in device memory, integrated in order, max_batch scans per GPU batch.  Scan s is
 * the points d_xyz[3*scan_offsets[s] .. 3*scan_offsets[s+1]) (offsets in points, host array of
 * n_scans+1) seen from origins[3*s .. 3*s+3) (host array).  d_xyz must stay valid and unchanged
 * until the next tsdf_sync (or read-out call) returns: a batch that overflowed the capacity is
 * re-run from it after growing (tsdf_params.max_bricks_hard). */
int tsdf_integrate_batch_device(tsdf_ctx* ctx, const float* d_xyz, const uint64_t* scan_offsets,
                                uint32_t n_scans, const double* origins);
/* ABI v6: the same with one pose (x, y, z, qx, qy, qz, qw) per scan (poses: host, 7 x n_scans). */
int tsdf_integrate_batch_device_pose(tsdf_ctx* ctx, const float* d_xyz,
                                     const uint64_t* scan_offsets, uint32_t n_scans,
                                     const double* poses);

/* Block until all queued work finished (growing capacity and re-running overflowed batches first,
 * see tsdf_params.max_bricks_hard); reports an overflow that could not be grown away as
 * TSDF_ENOMEM. */
int tsdf_sync(tsdf_ctx* ctx);

/* Dense read-out of voxels lo..hi-1 (voxel index coordinates, voxel i spans [i*vs, (i+1)*vs)),
 * x fastest: out[((z-lo2)*(hi1-lo1) + (y-lo1))*(hi0-lo0) + (x-lo0)].  Unobserved voxels, and
 * voxels outside the map's index domain (|i| >= 2^23 per axis), read (sdf_trunc, 0) — VDBFusion's
 * background values.  sdf / weight are host buffers.  ABI v10: int64 bounds; each
 * extent hi - lo must be below 2^31 and the box below 2^40 voxels (TSDF_EINVAL otherwise). */
int tsdf_query_dense(tsdf_ctx* ctx, const int64_t lo[3], const int64_t hi[3], float* sdf,
                     float* weight);

int tsdf_num_bricks(tsdf_ctx* ctx, uint64_t* n);

/* Copy every allocated brick out: coords[3*i..] = brick coordinates (voxel = 8*brick + local),
 * sdf/weight[512*i + (z*64 + y*8 + x)].  cap = capacity in bricks; *n_out = bricks written.
 * Returns TSDF_EOVERFLOW (and *n_out = required count) when cap is too small. */
int tsdf_export_bricks(tsdf_ctx* ctx, int32_t* coords, float* sdf, float* weight, uint64_t cap,
                       uint64_t* n_out);

/* Merge n unique bricks into the field: for every voxel with weight w_in > 0,
 * sdf <- (sdf*W + sdf_in*w_in) / (W + w_in), W <- W + w_in, or a plain copy where W == 0
 * (weighted-mean merge of partial fields; used for multi-GPU border bricks and for resuming
 * from an export).  With TSDF_SEM_VOXBLOX the merged weight is capped at max_weight, as Voxblox
 * caps every weight (its clamped update is order dependent, so a merge of Voxblox partial fields
 * is an approximation). */
int tsdf_import_bricks(tsdf_ctx* ctx, const int32_t* coords, const float* sdf, const float* weight,
                       uint64_t n);

int tsdf_get_stats(tsdf_ctx* ctx, tsdf_stats* out);
int tsdf_reset_stats(tsdf_ctx* ctx);
/* Record HIP events around every kernel (per-kind device time in tsdf_stats.kernel_ms). */
int tsdf_set_profiling(tsdf_ctx* ctx, int32_t on);
/* ABI v7: which launches profiling times.  Kinds whose bit (1 << TSDF_K_*) is in every_mask are
 * timed on every batch, the other kinds on every period-th batch (period 1: every batch; the
 * default is every kind on every batch).  A timed kernel records its own dispatch timestamps, which
 * costs the stream ~5 us per timed launch; bench.py times the dominant kernel on every batch and
 * samples the rest. */
int tsdf_set_profiling_period(tsdf_ctx* ctx, uint32_t every_mask, uint32_t period);

/* Append one JSON line per finished GPU batch to the file at `path` (NULL: stop), written at
 * tsdf_sync / read-outs (and every ~250 batches): batch id, scans, points, valid rays, (ray, brick)
 * pairs, voxel updates (sum over its scans of U_vox), dirty voxels, active and new bricks, pool
 * size, overflow bits, whether it committed (a batch re-run after a capacity growth reports
 * committed: false first), SURVEY §8d's algorithmic bytes, and with profiling on the per-kernel
 * times, path time and GB/s.  With max_batch = 1 every line is one scan (SURVEY §5 metrics). */
int tsdf_set_metrics_log(tsdf_ctx* ctx, const char* path);

/* Marching-cubes triangle mesh of the field (VDBFusion VDBVolume::extract_triangle_mesh; SURVEY
 * §8f.1): every 2x2x2 voxel cube whose 8 voxels are observed (W > 0 and W >= min_weight) is
 * meshed at S = 0.  Output: a triangle soup, 9 floats (3 vertices x, y, z, metres) per triangle,
 * ordered by brick (z, y, x), then cube, then case-table order.  tri == NULL: only *n_tri is set;
 * cap < *n_tri: TSDF_EOVERFLOW. */
int tsdf_extract_mesh(tsdf_ctx* ctx, float min_weight, float* tri, uint64_t cap, uint64_t* n_tri);

/* The generated marching-cubes case table (256 x 32 bytes: [case][0] = triangles, then 3 edge ids
 * per triangle; corner c = (c & 1, c >> 1 & 1, c >> 2 & 1); edges axis-major). */
int tsdf_mc_table(uint8_t* out);

/* ABI v6: marching-cubes case tables.  TSDF_MC_GENERATED: the table above (ambiguous faces paired
 * around their inside corners, so neighbouring cubes agree).  TSDF_MC_LORENSEN (ABI v8: the
 * literal data): the published Lorensen / Bourke triangle table that VDBFusion's
 * extract_triangle_mesh compiles in (include/tsdf_mc_tables.h), renumbered into this library's
 * corners and edges with its triangles' order and winding kept (ambiguous faces are split the
 * classic way, which can leave cracks).  TSDF_MC_LORENSEN_RULE: this library's restatement of the
 * classic ambiguity rule (round 3's TSDF_MC_LORENSEN), for comparison. */
#define TSDF_MC_GENERATED 0
#define TSDF_MC_LORENSEN 1
#define TSDF_MC_LORENSEN_RULE 2
#define TSDF_MC_TABLES 3
int tsdf_extract_mesh_table(tsdf_ctx* ctx, float min_weight, int32_t table, float* tri,
                            uint64_t cap, uint64_t* n_tri);
/* The case table `table` in tsdf_mc_table's layout (edges in this library's numbering). */
int tsdf_mc_table_of(int32_t table, uint8_t* out);

/* ---- Ouster sensor input ------------------------------------------------------
 * The reference's sensor path is the Ouster SDK (src/ouster/ouster-sdk/ouster_client): UDP lidar
 * packets -> LidarScan field images (parsing.cpp, lidar_scan.cpp ScanBatcher) -> xyz via the
 * make_xyz_lut LUT (lidar_scan.cpp:297-382, cartesian.h).  These entry points run that path on the
 * GPU so a frame's raw packets can go straight to tsdf_integrate_device. */
#define TSDF_OS_LEGACY 0
#define TSDF_OS_RNG19_RFL8_SIG16_NIR16 1
#define TSDF_OS_RNG19_RFL8_SIG16_NIR16_DUAL 2 /* first return only */
#define TSDF_OS_RNG15_RFL8_NIR8 3

typedef struct tsdf_os_format {
    uint32_t profile;            /* TSDF_OS_* (metadata data_format.udp_profile_lidar) */
    uint32_t pixels_per_column;  /* h */
    uint32_t columns_per_packet;
    uint32_t columns_per_frame;  /* w */
} tsdf_os_format;

/* Bytes of one lidar packet of this format (the UDP payload). */
int tsdf_os_packet_bytes(const tsdf_os_format* fmt, uint32_t* bytes);

/* Decode n_packets lidar packets of ONE frame (device memory, packed back to back) into staggered
 * h x w row-major u32 images (device; any may be NULL): column = measurement_id, columns with
 * status bit 0 clear are dropped, absent columns are 0 (the SDK's ScanBatcher).  Values are the
 * SDK's field values (RANGE in mm, masked / shifted per profile). */
int tsdf_os_decode_device(tsdf_ctx* ctx, const tsdf_os_format* fmt, const uint8_t* d_packets,
                          uint32_t n_packets, uint32_t* d_range, uint32_t* d_signal,
                          uint32_t* d_reflectivity, uint32_t* d_near_ir);

/* World points of a range image: xyz = r dir + off (dir, off: the xyz LUT, n x 3 float32, device;
 * r = 0 gives the sensor origin, dropped by the integrate), then x_world = pose * [xyz; 1] with
 * pose a 3x4 row-major matrix.  d_xyz: n x 3 float32 (device), ready for tsdf_integrate_device
 * with origin = the pose's translation. */
int tsdf_os_cartesian_device(tsdf_ctx* ctx, const uint32_t* d_range, uint64_t n, const float* d_dir,
                             const float* d_off, const double pose[12], float* d_xyz);

/* Azimuth sectors (multi-GPU sharding).  A ray's azimuth is taken as the fp32 pseudo-angle
 * a(dx, dy) in [0, 4) of (dx, dy) = (px - (float)ox, py - (float)oy) — monotone in the true
 * angle, exactly reproducible on host and GPU (one IEEE division, no trig):
 *     dy >= 0: dx >= 0 ? dy / (dx + dy) (0 when dx + dy == 0) : 1 - dx / (dy - dx)
 *     dy <  0: dx <  0 ? 2 - dy / (-dx - dy)                  : 3 + dx / (dx - dy)
 * Sector k starts at the pseudo-angle of yaw0 + 2 pi k / n (cos/sin in double, rounded to
 * float); sector k is [start_k, start_{k+1}) taken cyclically, so the sectors partition the
 * plane.  tsdf_sector_of gives the sector of one point (-1: zero-length / NaN). */
int32_t tsdf_sector_of(float px, float py, const double origin[3], double yaw0, uint32_t n_sectors);

/* Keep the points of sector `sector` (tsdf_sector_of's rule); packed to out_xyz (host, 3 f32 each). */
int tsdf_select_sector(const float* xyz, uint64_t n, const double origin[3], double yaw0,
                       uint32_t sector, uint32_t n_sectors, float* out_xyz, uint64_t* n_out);

/* ---- Border-brick reduce (multi-GPU read-out) ----------------------
 * Sector shards hold partial fields; VDBFusion's field is the weighted mean over all samples, so
 * the partial fields of a brick held by several ranks combine exactly (up to fp32 rounding).  The
 * reduce moves every shared brick's mass to its OWNER — the lowest rank holding it — over the
 * caller's collective (RCCL all-to-all over xGMI; the library does no communication):
 *   1. tsdf_brick_keys_device: this rank's brick keys -> all-gathered by the caller;
 *   2. tsdf_border_pack_device: this rank's bricks owned by a lower rank are packed as tiles
 *      (grouped by owner); ABI v9: they keep their mass until step 4;
 *   3. all_to_all of the tiles (caller), then tsdf_border_merge_device on every rank merges the
 *      received tiles into its bricks, sources in ascending rank order, by the rule of
 *      tsdf_import_bricks (weighted mean; copy where W == 0), after a snapshot of those bricks;
 *   4. (ABI v9) tsdf_border_commit_device on every rank, with commit = 1 only when the collective
 *      and EVERY rank's merge succeeded (the caller agrees on it, e.g. an all-reduce of the ranks'
 *      status): the sent bricks are reset to the background.  commit = 0 aborts: the merged bricks
 *      are restored from their snapshots and the sent bricks keep their mass, so every field is the
 *      one before the reduce, bit for bit -- a failed reduce neither loses nor double-counts mass.
 *      Between steps 2 and 4 (the reduce is open) the context refuses integrate and import calls.
 * Afterwards every brick's full mass sits on its owner (the others hold it at W = 0), so
 * integration may continue and the reduce may be repeated.  All buffers are DEVICE memory of the
 * context's GPU and must be ready when the call is made; the calls return after their own GPU work
 * finished.  Brick keys: 21 bits per axis, biased by 2^20 (x | y << 21 | z << 42). */
#define TSDF_TILE_WORDS 1028 /* u32 words per tile: 512 sdf f32, 512 weight f32, key lo, key hi, 0, 0 */
#define TSDF_MAX_WORLD 64

/* Keys of the context's bricks (device, cap entries); *n_out = bricks (TSDF_EOVERFLOW if > cap). */
int tsdf_brick_keys_device(tsdf_ctx* ctx, uint64_t* d_keys, uint64_t cap, uint64_t* n_out);

/* d_all_keys: world blocks of `stride` keys (device), block r = rank r's keys, counts[r] valid
 * (host array).  Packs the bricks of this context owned by a lower rank into d_send (device, rows
 * of TSDF_TILE_WORDS, grouped by owner rank ascending; cap_rows rows) and resets them.
 * send_counts[world] (host) receives the rows per destination; d_send == NULL only counts. */
int tsdf_border_pack_device(tsdf_ctx* ctx, const uint64_t* d_all_keys, const uint64_t* counts,
                            uint64_t stride, uint32_t world, uint32_t rank, uint32_t* d_send,
                            uint64_t cap_rows, uint64_t* send_counts);

/* Merge received tiles: d_recv (device) holds recv_counts[r] rows from each rank r, grouped by r
 * ascending.  Every tile's brick must exist here (it does on its owner). */
int tsdf_border_merge_device(tsdf_ctx* ctx, const uint32_t* d_recv, const uint64_t* recv_counts,
                             uint32_t world);

/* ABI v9: close the context's open border reduce: commit = 1 resets the bricks its pack sent;
 * commit = 0 restores the bricks its merges touched and keeps the sent ones.  No open reduce: a
 * no-op.  On a HIP error the reduce stays open (retry the call). */
int tsdf_border_commit_device(tsdf_ctx* ctx, int32_t commit);

/* ---- ABI v7: several GPUs in ONE process (SURVEY §8b's num_gpus / device_ids) ----------------
 * tsdf_create_sharded: n contexts, context k on device_ids[k] (NULL: device k) as azimuth sector k
 * of n (p's n_sectors / sector / device_id are overridden), into out[0..n).  ABI v8: peer access
 * is enabled between every pair of distinct devices that supports it (hipDeviceEnablePeerAccess),
 * so the input fan-out and the border reduce's tile copies run over xGMI; tsdf_stats.peer_mask
 * reports which contexts each one reaches directly.  Feed them with
 * tsdf_integrate_sectors (host clouds) or each with the full device scans; read out after
 * tsdf_border_reduce_local, which runs the three steps above among the n contexts of this process:
 * keys gathered on the host, each source's tiles copied to their owner's GPU with one peer copy
 * per (source, owner) pair.  Synchronous; *bricks_moved (may be NULL) = tiles merged.  Contexts of
 * different processes use the three device entry points with a collective instead. */
int tsdf_create_sharded(const tsdf_params* p, uint32_t n, const int32_t* device_ids,
                        tsdf_ctx** out);
/* ABI v9: transactional (every context packs without resetting, every owner snapshots before it
 * merges; any failure rolls every context back), so a failed call leaves the fields unchanged. */
int tsdf_border_reduce_local(tsdf_ctx* const* ctxs, uint32_t n, uint64_t* bricks_moved);

/* ---- ABI v9: marching cubes of a sector-sharded field (C5: 2 cm + mesh on N GPUs) -----------
 * After a border reduce every brick's mass sits on one context, but a cube on a brick's +x/+y/+z
 * faces also reads voxels of neighbour bricks, which another context may own.  Each context meshes
 * ITS bricks (a cube belongs to the brick of its min voxel, so every cube is meshed exactly once)
 * with a one-brick halo of the neighbours it lacks:
 *   tsdf_halo_keys_device   the keys of the +x/+y/+z neighbour bricks (7 per brick) of this
 *                           context's observed bricks that it does not observe itself (device,
 *                           sorted; TSDF_EOVERFLOW with *n_out = the count when cap is short)
 *   tsdf_halo_pack_device   on a holder: tiles (TSDF_TILE_WORDS rows: S, W, key) of the requested
 *                           bricks it observes, in any row order; *n_rows = tiles
 *   tsdf_extract_mesh_halo  tsdf_extract_mesh_table over this context's bricks, neighbours looked up
 *                           in the halo tiles first
 * The union of the contexts' soups is the mesh of the union field (tests/test_multigpu.py).
 * tsdf_extract_mesh_local runs all of it among the contexts of one process (border reduce, halo
 * exchange by peer copies, one mesh per context; soups concatenated in context order). */
int tsdf_halo_keys_device(tsdf_ctx* ctx, uint64_t* d_keys, uint64_t cap, uint64_t* n_out);
int tsdf_halo_pack_device(tsdf_ctx* ctx, const uint64_t* d_req, uint64_t n_req, uint32_t* d_send,
                          uint64_t cap_rows, uint64_t* n_rows);
int tsdf_extract_mesh_halo(tsdf_ctx* ctx, float min_weight, int32_t table, const uint32_t* d_halo,
                           uint64_t n_halo, float* tri, uint64_t cap, uint64_t* n_tri);
int tsdf_extract_mesh_local(tsdf_ctx* const* ctxs, uint32_t n, float min_weight, int32_t table,
                            float* tri, uint64_t cap, uint64_t* n_tri);

#ifdef __cplusplus
}
#endif
#endif /* TSDF_HIP_H */
