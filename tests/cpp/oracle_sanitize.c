/* oracle_sanitize.c -- drives the CPU oracle (oracle/tsdf_oracle.c, test infrastructure) through
 * its whole C-ABI surface so it can be built with -fsanitize=address,undefined and with
 * -fsanitize=thread (oracle/Makefile `sanitize`; tests/test_sanitize.py runs both; SURVEY §5
 * "Race detection / sanitizers").  Exercised:
 *   - every semantics, serial vs the partitioned multi-threaded scan-fused mode (bit for bit),
 *     the sequential and VDB-literal modes, Voxblox merged bundling, space carving;
 *   - the exact fixed-point sums at their extremes: Voxblox 1/z^2 weights capped at 2^16 on
 *     thousands of points in one voxel, points on voxel faces, far coordinates;
 *   - import / export / query, marching cubes (every table), the border-reduce transaction
 *     (commit and abort), the one-process sharded calls and the sharded mesh.
 * Input: argv[1], scans as u64 n_scans, then per scan u64 n, f64 origin[3], f32 xyz[3 n].
 * Prints "ok" and exits 0; any sanitizer report aborts (-fno-sanitize-recover=all). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/tsdf_hip.h"

int tsdf_oracle_set_mode(tsdf_ctx* c, int mode);
int tsdf_oracle_set_threads(tsdf_ctx* c, int n);
uint64_t tsdf_oracle_num_voxels(const tsdf_ctx* c);
int tsdf_oracle_export_voxels(const tsdf_ctx* c, int32_t* ijk, float* sdf, float* w, uint64_t cap,
                              uint64_t* n_out);

typedef struct { uint64_t n; double o[3]; float* xyz; } scan_t;

static int fails = 0;
#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fprintf(stderr, "\n");                        \
            fails++;                                      \
        }                                                 \
    } while (0)
#define OK(expr) CHECK((expr) == TSDF_OK, "%s", #expr)

typedef struct { uint64_t n; int32_t* ijk; float *s, *w; } field_t;

static field_t field(const tsdf_ctx* c) {
    field_t f;
    f.n = tsdf_oracle_num_voxels(c);
    f.ijk = (int32_t*)malloc((f.n + 1) * 12);
    f.s = (float*)malloc((f.n + 1) * 4);
    f.w = (float*)malloc((f.n + 1) * 4);
    uint64_t got = 0;
    OK(tsdf_oracle_export_voxels(c, f.ijk, f.s, f.w, f.n, &got));
    return f;
}

static int same(field_t a, field_t b) {
    return a.n == b.n && !memcmp(a.ijk, b.ijk, a.n * 12) && !memcmp(a.s, b.s, a.n * 4) &&
           !memcmp(a.w, b.w, a.n * 4);
}

static void drop(field_t f) { free(f.ijk); free(f.s); free(f.w); }

static tsdf_params params(int sem) {
    tsdf_params p;
    tsdf_default_params(&p);
    p.semantics = sem;
    p.max_range = 100.0;
    return p;
}

static tsdf_ctx* make(const tsdf_params* p) {
    tsdf_ctx* c = NULL;
    OK(tsdf_create(p, &c));
    return c;
}

static void pose_of(const scan_t* s, int k, double q[7]) {
    q[0] = s->o[0]; q[1] = s->o[1]; q[2] = s->o[2];
    q[3] = 0.0; q[4] = 0.05 * k; q[5] = sin(0.1 * k); q[6] = 1.0;  /* tilted: 1/z^2 matters */
}

/* serial vs threaded, one semantics / method */
static void modes(const scan_t* sc, int ns, int sem, int method, int carving, int threads) {
    tsdf_params p = params(sem);
    p.voxblox_method = method;
    p.space_carving = carving;
    if (carving) p.max_range = 30.0;
    tsdf_ctx* a = make(&p);
    tsdf_ctx* b = make(&p);
    OK(tsdf_oracle_set_threads(b, threads));
    for (int k = 0; k < ns; k++) {
        double q[7];
        pose_of(&sc[k], k, q);
        OK(tsdf_integrate_pose(a, sc[k].xyz, sc[k].n, 12, 0, 0, q));
        OK(tsdf_integrate_pose(b, sc[k].xyz, sc[k].n, 12, 0, 0, q));
    }
    field_t fa = field(a), fb = field(b);
    CHECK(fa.n > 1000 && same(fa, fb), "threaded != serial (sem %d method %d carving %d): %llu %llu",
          sem, method, carving, (unsigned long long)fa.n, (unsigned long long)fb.n);
    drop(fa); drop(fb);
    tsdf_destroy(a);
    tsdf_destroy(b);
}

/* Voxblox 1/z^2 at its cap: thousands of points in one voxel close to the sensor plane, plus
 * points on voxel faces and at far coordinates (the int64 fixed-point sums' extremes) */
static void extremes(void) {
    tsdf_params p = params(TSDF_SEM_VOXBLOX);
    p.max_weight = 1e30f;  /* only TSDF_W0_CAP bounds a sample */
    tsdf_ctx* c = make(&p);
    const int n = 6000;
    float* xyz = (float*)malloc(n * 12);
    for (int i = 0; i < n; i++) {  /* ~1e-5 m off the sensor's x-y plane: 1/z^2 ~ 1e10, capped */
        xyz[3 * i] = 0.4f + 1e-6f * (float)(i % 7);
        xyz[3 * i + 1] = 0.3f;
        xyz[3 * i + 2] = 1e-5f;
    }
    const double q[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0};
    for (int r = 0; r < 3; r++) OK(tsdf_integrate_pose(c, xyz, n, 12, 0, 0, q));
    field_t f = field(c);
    CHECK(f.n > 0, "capped weights integrated nothing");
    for (uint64_t i = 0; i < f.n; i++) CHECK(isfinite(f.s[i]) && f.w[i] > 0.0f, "bad voxel");
    drop(f);
    tsdf_destroy(c);
    /* VDBFusion f64 / fp32: rays onto voxel faces and corners, and far from the origin */
    for (int sem = 0; sem <= 2; sem += 2) {
        tsdf_params pv = params(sem);
        pv.max_range = 1e7;
        tsdf_ctx* v = make(&pv);
        float pts[8][3] = {{0.05f, 0.1f, 0.15f}, {1.0f, 1.0f, 1.0f}, {-0.05f, 2.5f, -0.1f},
                           {100000.0f, 3.0f, 2.0f}, {-99999.95f, -0.05f, 0.0f},
                           {3.0f, 0.0f, 0.0f}, {0.0f, 3.0f, 0.0f}, {0.0f, 0.0f, 3.0f}};
        const double o[3] = {0.0, 0.0, 0.0};
        const double o2[3] = {99990.0, 1.0, 1.0};
        OK(tsdf_integrate(v, pts, 8, 12, 0, 0, o));
        OK(tsdf_integrate(v, pts, 8, 12, 0, 0, o2));
        CHECK(tsdf_oracle_num_voxels(v) > 10, "face rays integrated nothing");
        tsdf_destroy(v);
    }
    free(xyz);
}

static void readout(const scan_t* sc) {
    tsdf_params p = params(TSDF_SEM_VDBFUSION_F64);
    tsdf_ctx* a = make(&p);
    OK(tsdf_integrate(a, sc[0].xyz, sc[0].n, 12, 0, 0, sc[0].o));
    uint64_t nb = 0, got = 0;
    OK(tsdf_num_bricks(a, &nb));
    int32_t* co = (int32_t*)malloc(nb * 12 + 12);
    float* s = (float*)malloc(nb * 2048 + 4);
    float* w = (float*)malloc(nb * 2048 + 4);
    OK(tsdf_export_bricks(a, co, s, w, nb, &got));
    CHECK(tsdf_export_bricks(a, co, s, w, nb ? nb - 1 : 0, &got) == TSDF_EOVERFLOW, "export cap");
    tsdf_ctx* b = make(&p);
    OK(tsdf_import_bricks(b, co, s, w, nb));
    field_t fa = field(a), fb = field(b);
    CHECK(same(fa, fb), "import != export");
    drop(fa); drop(fb);
    const int64_t lo[3] = {-40, -40, -10}, hi[3] = {40, 40, 10};
    float* qs = (float*)malloc(80 * 80 * 20 * 4);
    float* qw = (float*)malloc(80 * 80 * 20 * 4);
    OK(tsdf_query_dense(a, lo, hi, qs, qw));
    for (int t = 0; t < TSDF_MC_TABLES; t++) {
        uint64_t nt = 0;
        OK(tsdf_extract_mesh_table(a, 0.0f, t, NULL, 0, &nt));
        float* tri = (float*)malloc(nt * 36 + 36);
        OK(tsdf_extract_mesh_table(a, 0.0f, t, tri, nt, &nt));
        if (nt) CHECK(tsdf_extract_mesh_table(a, 0.0f, t, tri, nt - 1, &nt) == TSDF_EOVERFLOW, "mesh cap");
        free(tri);
    }
    /* sequential and literal modes on the same scan */
    for (int mode = 1; mode <= 2; mode++) {
        tsdf_ctx* m = make(&p);
        OK(tsdf_oracle_set_mode(m, mode));
        OK(tsdf_integrate(m, sc[0].xyz, sc[0].n, 12, 0, 0, sc[0].o));
        CHECK(tsdf_oracle_num_voxels(m) > 1000, "mode %d integrated nothing", mode);
        tsdf_destroy(m);
    }
    free(co); free(s); free(w); free(qs); free(qw);
    tsdf_destroy(a);
    tsdf_destroy(b);
}

/* the border transaction, the sharded calls and the sharded mesh on 3 sector contexts */
static void sharded(const scan_t* sc, int ns) {
    enum { N = 3 };
    tsdf_params p = params(TSDF_SEM_VDBFUSION_F64);
    p.sector_yaw0 = 0.3;
    tsdf_ctx* c[N];
    OK(tsdf_create_sharded(&p, N, NULL, c));
    for (int k = 0; k < ns; k++) {
        double q[7];
        pose_of(&sc[k], k, q);
        OK(tsdf_integrate_sectors(c, N, sc[k].xyz, sc[k].n, 12, 0, 0, q));
        OK(tsdf_integrate_sectors_origin(c, N, sc[k].xyz, sc[k].n, 12, 0, 0, sc[k].o));
    }
    field_t before[N];
    for (int r = 0; r < N; r++) before[r] = field(c[r]);
    /* a reduce by hand, then aborted: every field as before */
    uint64_t counts[N], stride = 1;
    for (int r = 0; r < N; r++) {
        OK(tsdf_num_bricks(c[r], &counts[r]));
        if (counts[r] > stride) stride = counts[r];
    }
    uint64_t* all = (uint64_t*)malloc(N * stride * 8);
    for (uint64_t i = 0; i < N * stride; i++) all[i] = ~0ull;
    for (int r = 0; r < N; r++) OK(tsdf_brick_keys_device(c[r], all + r * stride, stride, &counts[r]));
    uint32_t* send[N];
    uint64_t sc_[N][N];
    for (int r = 0; r < N; r++) {
        send[r] = (uint32_t*)malloc((counts[r] + 1) * TSDF_TILE_WORDS * 4);
        OK(tsdf_border_pack_device(c[r], all, counts, stride, N, r, send[r], counts[r], sc_[r]));
    }
    for (int d = 0; d < N; d++) {
        uint64_t rc[N], tot = 0;
        for (int r = 0; r < N; r++) { rc[r] = sc_[r][d]; tot += rc[r]; }
        uint32_t* recv = (uint32_t*)malloc((tot + 1) * TSDF_TILE_WORDS * 4);
        uint64_t row = 0;
        for (int r = 0; r < N; r++) {
            uint64_t off = 0;
            for (int e = 0; e < d; e++) off += sc_[r][e];
            memcpy(recv + row * TSDF_TILE_WORDS, send[r] + off * TSDF_TILE_WORDS, rc[r] * TSDF_TILE_WORDS * 4);
            row += rc[r];
        }
        OK(tsdf_border_merge_device(c[d], recv, rc, N));
        free(recv);
    }
    CHECK(tsdf_integrate(c[0], sc[0].xyz, sc[0].n, 12, 0, 0, sc[0].o) == TSDF_EINVAL, "open reduce took a scan");
    for (int r = 0; r < N; r++) OK(tsdf_border_commit_device(c[r], 0));
    for (int r = 0; r < N; r++) {
        field_t f = field(c[r]);
        CHECK(same(f, before[r]), "abort did not restore rank %d", r);
        drop(f);
        drop(before[r]);
        free(send[r]);
    }
    free(all);
    uint64_t moved = 0, nt = 0;
    OK(tsdf_border_reduce_local(c, N, &moved));
    CHECK(moved > 10, "no border bricks moved");
    OK(tsdf_extract_mesh_local(c, N, 0.0f, TSDF_MC_LORENSEN, NULL, 0, &nt));
    float* tri = (float*)malloc(nt * 36 + 36);
    OK(tsdf_extract_mesh_local(c, N, 0.0f, TSDF_MC_LORENSEN, tri, nt, &nt));
    CHECK(nt > 100, "sharded mesh is empty");
    free(tri);
    for (int r = 0; r < N; r++) tsdf_destroy(c[r]);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint64_t ns = 0;
    if (fread(&ns, 8, 1, f) != 1 || ns == 0 || ns > 64) return 2;
    scan_t* sc = (scan_t*)calloc(ns, sizeof(scan_t));
    for (uint64_t k = 0; k < ns; k++) {
        if (fread(&sc[k].n, 8, 1, f) != 1 || fread(sc[k].o, 8, 3, f) != 3) return 2;
        sc[k].xyz = (float*)malloc(sc[k].n * 12 + 12);
        if (fread(sc[k].xyz, 12, sc[k].n, f) != sc[k].n) return 2;
    }
    fclose(f);
    const int threads = argc > 2 ? atoi(argv[2]) : 4;
    const char* what = argc > 3 ? argv[3] : "all";
    const int all = !strcmp(what, "all");
    if (all || !strcmp(what, "threads")) {
        modes(sc, (int)ns, TSDF_SEM_VDBFUSION_F64, TSDF_VB_SIMPLE, 0, threads);
        modes(sc, (int)ns, TSDF_SEM_VDBFUSION, TSDF_VB_SIMPLE, 0, threads);
        modes(sc, (int)ns, TSDF_SEM_VOXBLOX, TSDF_VB_SIMPLE, 0, threads);
    }
    if (all) {
        modes(sc, (int)ns, TSDF_SEM_VOXBLOX, TSDF_VB_MERGED, 0, threads);
        modes(sc, 1, TSDF_SEM_VDBFUSION, TSDF_VB_SIMPLE, 1, threads);
        extremes();
        readout(sc);
        sharded(sc, (int)ns);
    }
    for (uint64_t k = 0; k < ns; k++) free(sc[k].xyz);
    free(sc);
    if (fails) {
        fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    printf("ok\n");
    return 0;
}
