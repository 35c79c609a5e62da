// simaps.hip -- MI355X (gfx950) kernels of the Spatial Intention Maps observation path.
//
// One workgroup (1024 threads = 16 waves) renders one agent-state stack end to end with every
// intermediate resident in LDS (~158 KiB, one workgroup per CU):
//
//   0. params    per-robot stamp rotations (scipy rotate geometry, fp64) and <= 32x32 rotated
//                mask bit tiles (Mapper._create_global_robot_map, envs.py:2251-2276).
//   1. cspace    OccupancyMap.update (envs.py:2453-2454): 1 - max(1 - room_mask,
//                binary_dilation(occ, disk(r))) inside the room rect; occupancy rows staged
//                through LDS, turned into bit rows by wave ballots, disk dilation as OR of
//                shifted bit rows.
//   2. snap      OccupancyMap._closest_valid_cspace_indices (envs.py:2523-2524) =
//                scipy distance_transform_edt(return_indices) evaluated at the <= 2 query pixels
//                with scipy's own separable Voronoi tie-breaking (column pass, then one lane).
//   3. SSSP      GridGraph._spfa (pyx:69-114) from the <= 2 snapped sources as rounds of four
//                concurrent directional sweeps per source (one wave each: down / up / right /
//                left; lane = column or row, DPP lane shifts carry the diagonal neighbours).
//                The float32 fixpoint is unique (dist[v] = min over paths of the left-fold f32
//                sum), so any schedule that runs to convergence is bit-identical to the
//                reference's SPFA.  WHILE the sweep waves run, the other waves render:
//   4. render    Mapper.get_state (envs.py:2068-2113) channels that do not need distances:
//                overhead + robot (robot stamps OR-ed into a 136x136 one-hot code map in LDS,
//                then one gather per output pixel through the scipy order-0 rotate index rule),
//                history / intention lines rasterised into an LDS tile (closed-form Bresenham,
//                fp64 linspace ramp, atomicMax) and grey-dilated at sample time, intention
//                channels.
//   5. distance  after the sweeps converge, all 16 waves render the distance channels
//                (Euclidean-to-receptacle, shortest-path maps with the reference's max / scale
//                / min-subtract order).
//
// HBM traffic per stack: the occupancy window (room rect + r halo, bytes), the overhead window
// gathered through L2 (<= 136^2 f32 footprint), the state write (96*96*C f32).  No intermediate
// map ever leaves the CU.
//
// Diagnostic-only build macros (never the product): SIMAPS_PHASE_STAMPS / SIMAPS_LIGHT_STAMPS
// (per-phase s_memrealtime stamps, tools/phase_profile.py, `make prof`), SIMAPS_DIAG_FLAG_TIMEOUT
// (the fault-path test build, `make diag`).  The round-1/2 ablation variants (sweeps or render
// alone, no gathers / raster / stores, issue-priority variants) were measured and removed; their
// results are in DESIGN.md.
//
// Compiled with -ffp-contract=off: every fp32/fp64 operation rounds exactly like the reference
// (see geom.h for the one explicit fma).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "geom.h"
#include "mixed.h"
#include "simaps.h"

using namespace simaps;

namespace {

constexpr int NT = 1024;
#if defined(SIMAPS_PHASE_STAMPS) || defined(SIMAPS_LIGHT_STAMPS)
// Diagnostic builds only (libsimaps_prof.so): per-workgroup s_memrealtime (100 MHz) stamps.
// SIMAPS_LIGHT_STAMPS: only a few stamps and no added barriers (code as close to the product's as a
// stamp build gets).
constexpr int MAX_STAMP_WG = 8192, NSTAMP = 80;
__device__ unsigned long long g_stamps[MAX_STAMP_WG * NSTAMP];
#ifdef SIMAPS_LIGHT_STAMPS
#ifdef SIMAPS_LIGHT_SET
#define STAMP_ON(k) (SIMAPS_LIGHT_SET(k))
#else
#define STAMP_ON(k) ((k) == 0 || (k) == 7 || (k) == 8 || (k) == 11 || (k) == 13 || (k) == 60 || (k) == 61 || (k) == 62)
#endif
#define STAMP_BAR()
#else
#define STAMP_ON(k) true
#define STAMP_BAR() lds_barrier()
#endif
// (a barrier first, so a stamp marks the moment the SLOWEST wave finished the previous phase)
#define STAMP(k)                                                                                 \
    do {                                                                                         \
        if (STAMP_ON(k)) {                                                                       \
            STAMP_BAR();                                                                         \
            if (threadIdx.x == 0 && blockIdx.x < MAX_STAMP_WG)                                   \
                g_stamps[blockIdx.x * NSTAMP + (k)] = __builtin_amdgcn_s_memrealtime();          \
        }                                                                                        \
    } while (0)
#define STAMP_NB(k)                                                                              \
    do {                                                                                         \
        if (STAMP_ON(k) && (threadIdx.x & 63) == 0 && blockIdx.x < MAX_STAMP_WG)                 \
            g_stamps[blockIdx.x * NSTAMP + (k)] = __builtin_amdgcn_s_memrealtime();              \
    } while (0)
#define STAMP_VAL(k, v) /* a counter instead of a time (e.g. the SPFA's pops) */             \
    do {                                                                                         \
        if (STAMP_ON(k) && blockIdx.x < MAX_STAMP_WG)                                            \
            g_stamps[blockIdx.x * NSTAMP + (k)] = (unsigned long long)(v);                       \
    } while (0)
#define STAMP_CLK(k) /* shader-clock counter (s_memtime): with a realtime stamp, the clock rate */  \
    do {                                                                                         \
        if (STAMP_ON(k) && (threadIdx.x & 63) == 0 && blockIdx.x < MAX_STAMP_WG)                 \
            g_stamps[blockIdx.x * NSTAMP + (k)] = __builtin_amdgcn_s_memtime();                  \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#define STAMP_NB(k) \
    do {            \
    } while (0)
#define STAMP_VAL(k, v) \
    do {                \
    } while (0)
#define STAMP_CLK(k) \
    do {             \
    } while (0)
#endif
constexpr int MAX_SEG = 128;     // intention / history segments per agent
constexpr int RBLK = (CROP + 7) / 8;  // 8 x 8 blocks per crop side (robot sets, render_maps)
constexpr int SEG_PER_ROBOT = SIMAPS_MAX_PATH - 1;
constexpr int MAX_ROWS = 112;    // room rect rows (bit-row arrays)
constexpr int RMAX = 7;  // floor(RADIUS * 96) <= 6 for every robot class (envs.py:2421)
static_assert(2 * RMAX < 32, "cspace window funnel shifts");
constexpr int WIN_WORDS = 3;     // occupancy window row: up to 192 bits
constexpr int MAX_WIN_ROWS = MAX_ROWS + 16;
constexpr unsigned INF_BITS = 0x7f800000u;
constexpr float SQRT2F = 1.41421354f;  // float(np.sqrt(2)) (pyx:31-32)

struct B128 {
    uint64_t lo, hi;
};
__device__ __forceinline__ B128 b_or(B128 a, B128 b) { return {a.lo | b.lo, a.hi | b.hi}; }
__device__ __forceinline__ B128 b_and(B128 a, B128 b) { return {a.lo & b.lo, a.hi & b.hi}; }
__device__ __forceinline__ B128 b_shl1(B128 a) { return {a.lo << 1, (a.hi << 1) | (a.lo >> 63)}; }
__device__ __forceinline__ B128 b_shr1(B128 a) { return {(a.lo >> 1) | (a.hi << 63), a.hi >> 1}; }
__device__ __forceinline__ bool b_test(const B128 &a, int c)
{
    return c < 64 ? (a.lo >> c) & 1 : (a.hi >> (c - 64)) & 1;
}
__device__ __forceinline__ B128 b_mask(int w)
{
    B128 m;
    m.lo = w >= 64 ? ~0ull : ((1ull << w) - 1);
    m.hi = w >= 128 ? ~0ull : (w > 64 ? ((1ull << (w - 64)) - 1) : 0ull);
    return m;
}
// bits [o, o + 128) of a 3-word row, 0 <= o < 64
__device__ __forceinline__ B128 win_get(const uint64_t *row, int o)
{
    B128 r;
    if (o == 0) {
        r.lo = row[0];
        r.hi = row[1];
    } else {
        r.lo = (row[0] >> o) | (row[1] << (64 - o));
        r.hi = (row[1] >> o) | (row[2] << (64 - o));
    }
    return r;
}
__device__ __forceinline__ void b_atomic_or(B128 *dst, B128 v)
{
    unsigned *w = reinterpret_cast<unsigned *>(dst);
    if ((unsigned)v.lo) atomicOr(w + 0, (unsigned)v.lo);
    if ((unsigned)(v.lo >> 32)) atomicOr(w + 1, (unsigned)(v.lo >> 32));
    if ((unsigned)v.hi) atomicOr(w + 2, (unsigned)v.hi);
    if ((unsigned)(v.hi >> 32)) atomicOr(w + 3, (unsigned)(v.hi >> 32));
}

// Workgroup barrier that orders LDS only.  __syncthreads() also waits vmcnt(0), i.e. for every
// outstanding global STORE of the wave -- no barrier in this file protects global memory, and that
// wait would expose the output write latency at every phase boundary.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------------------------------------------------------------------------
// Wave groups: the workgroup splits into SSSP-sweep waves and render waves that run concurrently.
// A group of fewer than 16 waves synchronises through an LDS barrier (lane 0 of each wave arrives
// on a counter; the last one bumps a generation word the others poll with s_sleep; bounded spin).
// ------------------------------------------------------------------------------------------------
struct Group {
    int t, n;           // thread index within the group, threads in the group
    unsigned *bar;      // nullptr: the whole workgroup (__syncthreads)
    int nw;             // waves in the group
    __device__ __forceinline__ void sync() const
    {
        if (!bar) {
            lds_barrier();
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        // relaxed LDS atomics, ordered by the local-only fences around them: acquire / release
        // orderings on the atomics themselves would also wait for every outstanding GLOBAL access
        // of the wave (vmcnt(0)), exposing the render group's gather / store latency at each sync
        if ((threadIdx.x & 63) == 0) {
            const unsigned g = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const unsigned arrived = __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (arrived == (unsigned)nw - 1) {
                __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(&bar[1], g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                unsigned spins = 0;
                while (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == g) {
                    __builtin_amdgcn_s_sleep(1);
#ifdef SIMAPS_DIAG_FLAG_TIMEOUT  // diagnostic build (tests/test_gpu_faults.py): raise the timeout
                    // flag at its real site on the first spin but keep waiting, so the output stays valid
                    if (spins == 0) __hip_atomic_store(&bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
                    if (++spins > (1u << 22)) {  // ~0.1 s: never in a correct run; flag (-> the fault
                        // word, SIMAPS_FAULT_TIMEOUT, at the kernel's end) and fall through
                        __hip_atomic_store(&bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        break;
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
};

__device__ __forceinline__ Group whole_wg() { return Group{(int)threadIdx.x, 1024, nullptr, 16}; }

constexpr int SIMAPS_NFAULT = 3;  // SIMAPS_FAULT_* bits

// Always-on fault reporting (include/simaps.h SIMAPS_FAULT_*): one thread per workgroup, after the
// kernel's last LDS barrier, ORs the conditions that invalidate its output into the process-wide
// host-mapped fault word.  `desc` holds SIMAPS_FAULT_DESCRIPTOR if a descriptor was clamped.
__device__ __forceinline__ unsigned group_faults(const unsigned (&bar)[4][4], int rounds, int nsrc)
{
    unsigned f = (bar[0][2] | bar[1][2] | bar[2][2] | bar[3][2]) ? SIMAPS_FAULT_TIMEOUT : 0u;
    if (nsrc > 0 && rounds >= (1 << 20)) f |= SIMAPS_FAULT_ROUNDS;
    return f | (bar[0][3] ? SIMAPS_FAULT_DESCRIPTOR : 0u);
}
__device__ __forceinline__ void post_faults(unsigned *fault, unsigned f)
{
    // fault[k] = 1 for bit k: plain system-scope vector stores into fine-grained host memory (no
    // PCIe atomics needed; concurrent writers store the same value); only in a faulting workgroup,
    // i.e. never in a correct run
    if (fault)
        for (int k = 0; k < SIMAPS_NFAULT; k++)
            if (f & (1u << k)) __hip_atomic_store(fault + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A workgroup's own LDS fault word: waves that do not meet at a barrier (the overlapped path kernel's
// SPFA wave beside its sweep waves) may set bits at the same time, so every writer ORs atomically.
__device__ __forceinline__ void fault_or(unsigned &word, unsigned f)
{
    __hip_atomic_fetch_or(&word, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ------------------------------------------------------------------------------------------------
// LDS layout
// ------------------------------------------------------------------------------------------------
struct RobotP {
    double c, s, f0, f1;  // stamp rotation (angle = degrees(h) - 90, envs.py:2266)
    double x, y, tx, ty;
    int S0, S1, st_i, st_j;  // stamp shape, placement (pixel - S // 2, envs.py:2272)
    int type, lifting, idle, group;
    int bi0, bi1, bj0, bj1;  // global-pixel box outside which the rotated mask is surely 0 (16-B aligned)
    int tpi, tpj;            // target end-effector pixel
    unsigned code0;          // robot-code bits of a class-mask pixel (robot_bits)
    float seg_val;
};

struct Seg {
    double start, step, stop;
    int si, sj, ti, tj;
    int n, last, dr, dc;
};

struct Shared {
    Rot rot;             // local map rotation (angle = 90 - degrees(h), envs.py:2203)
    int pi, pj;          // agent pixel
    int nr, me, env, has_rec;
    int h, w, i0, j0, r;
    int nsrc;
    int src_q[2][2], src_s[2][2], src_ok[2];
    int sp_slot[2];      // which dist buffer each sp channel uses (-1 = off)
    float dmax[2];
    float unreach[2];    // scaled value of unreachable / outside cells
    int flag[2];
    int rounds;          // SSSP rounds to convergence (-1: cap hit)
    int nseg;
    int seg_robot_cnt[SIMAPS_MAX_ROBOTS];
    int order[SIMAPS_MAX_ROBOTS];
    float red[3][16];
    float nonsp[2 * SIMAPS_MAX_ROBOTS];
    RobotP rob[SIMAPS_MAX_ROBOTS];
    unsigned bar[4][4];              // group barriers {count, generation, timeout, -}: [0] sweep track, [1] render,
                                     // [2 + s] source s's sweep waves (rounds)
    int changed[2][3];               // per source, rotating per-round "some sweep improved a cell" flags
    uint64_t dirty[2][4][2];         // per source and sweep direction: lines (bit L - 1) to relax again
    int scratch_free;                // the cspace scratch may be reused as the raster tile
    uint32_t mwin[5 * 24 + 20];      // robot mask windows: [5][24] bit rows + [5][4] ints (stamp tiles)
    Seg seg[MAX_SEG];
    double seglen[MAX_SEG];          // seg_geom -> seg_ramp: each segment's scaled length
};

// SSSP scratch (aliases the raster tile, which is only used after the SSSP phase)
struct SsspScratch {
    uint64_t win[MAX_WIN_ROWS][WIN_WORDS];
    B128 freeb[MAX_ROWS];
    B128 dtab[RMAX + 1][MAX_WIN_ROWS];  // window row dilated horizontally by +-j, rect columns (build_cspace)
};

constexpr int align16(int x) { return (x + 15) & ~15; }
constexpr int OFF_DIST = align16((int)sizeof(Shared));
constexpr int DIST_FLOATS = SIMAPS_MAX_ROOM_CELLS;  // (h + 2) * pitch, pitch = (w + 2) | 1
constexpr int OFF_UNION = OFF_DIST + align16(2 * DIST_FLOATS * 4);
constexpr int TILE_BYTES = TILE * TILE * 4;
constexpr int UNION_BYTES = align16((int)sizeof(SsspScratch) > TILE_BYTES ? (int)sizeof(SsspScratch) : TILE_BYTES);
constexpr int LDS_BYTES = OFF_UNION + UNION_BYTES;
// The crop's robot-code map (u8 per crop pixel + a zero guard for outside pixels), built by the
// stamps phase and read by the overhead / robot channels before the first raster pass: it shares the
// union with the sweep track's scratch (disjoint offsets) and with the raster tile (later in time).
constexpr int OFF_CMAP = OFF_UNION + align16((int)sizeof(SsspScratch));
// early_tile: the raster tile's first SCRATCH_Q 16-byte words overlap the cspace scratch (zeroed by
// the sweep track once it is released); the render track zeroes the rest at its start
constexpr int SCRATCH_Q = align16((int)sizeof(SsspScratch)) / 16;
static_assert(SCRATCH_Q <= TILE * TILE / 4, "scratch inside the tile");
constexpr int CMAP_BYTES = align16(CROP * CROP + 16);
static_assert(OFF_CMAP + CMAP_BYTES <= OFF_UNION + UNION_BYTES, "code map fits the union");
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
// distance phase: a cval pixel's cell byte offset (16 bits, 4-aligned, past every real cell; its
// read stays inside the LDS allocation and is discarded)
constexpr unsigned CVAL_OFF = 0xfffcu;
static_assert(DIST_FLOATS * 4 <= (int)CVAL_OFF && OFF_DIST + DIST_FLOATS * 4 + (int)CVAL_OFF + 4 <= LDS_BYTES,
              "distance-phase cell offsets fit 16 bits, the cval read stays in LDS");
static_assert(LW * LW * 4 <= TILE_BYTES, "sample-index + cell tables fit the raster tile");
typedef float f32x2 __attribute__((ext_vector_type(2)));
static_assert(offsetof(RobotP, bi0) % 16 == 0 && sizeof(RobotP) % 16 == 0, "RobotP box loads as one b128");

// ------------------------------------------------------------------------------------------------
// Block reductions (16 waves)
// ------------------------------------------------------------------------------------------------
// DPP within each 16-lane row (quad swaps, half-row and row mirrors), then the 4 row results by
// readlane: no LDS round trips (ds_bpermute) and a wave-uniform result.  NaN-free inputs only.
#define WAVE_REDUCE_F32(v, OP)                                                                          \
    do {                                                                                                \
        v = OP(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xf, 0xf, false)));  \
        v = OP(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xf, 0xf, false)));  \
        v = OP(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xf, 0xf, false))); \
        v = OP(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xf, 0xf, false))); \
        const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));                \
        const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));               \
        const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));               \
        const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));               \
        v = OP(OP(r0, r1), OP(r2, r3));                                                                 \
    } while (0)
__device__ __forceinline__ float wave_min(float v)
{
    WAVE_REDUCE_F32(v, fminf);
    return v;
}
__device__ __forceinline__ float wave_max(float v)
{
    WAVE_REDUCE_F32(v, fmaxf);
    return v;
}

// ------------------------------------------------------------------------------------------------
// Phase: occupancy window -> free-cell bit rows (cspace inside the room rect)
// ------------------------------------------------------------------------------------------------
// occ: the agent's occupancy map [H, W] (nonzero = obstacle).  r = disk radius (<= RMAX).
// The window loads are issued first thing by the group that builds the cspace (cspace_load, for the
// largest radius, so they need no robot descriptor) and land in registers.
// RN(v / 96) for v == 0 or 1 <= v < 2^32 (every SPFA distance): the reciprocal product with one FMA
// correction, exhaustively checked against IEEE division over that range (the general division is
// ~10 instructions)
__device__ __forceinline__ float div96(float v)
{
    const float r = 1.0f / 96.0f;
    const float q0 = v * r;
    return fmaf(fmaf(-q0, 96.0f, v), r, q0);
}

// distance-array pitch: (w + 2) | 1 floats (odd: column-wise sweeps hit at most 2-way bank conflicts)
__device__ __forceinline__ int sssp_pitch(int w) { return (w + 2) | 1; }

// ---- receptacle distance cache (simaps_debug.rec_cache, simaps_sp_lookup) -------------------------
// One record per map slot: int4 header {1, receptacle snapped to a free cell, h, w}, then the room
// rect's distance array as the sweeps leave it: (h + 2) x pitch float32, border and blocked cells
// -inf, free unreachable cells +inf (so a cell is free iff its value is above -inf).
constexpr int REC_HDR = 16;
__host__ __device__ __forceinline__ int rec_cache_bytes(int h, int w)
{
    return (REC_HDR + (h + 2) * ((w + 2) | 1) * 4 + 255) & ~255;
}
// Threads t of n write slot record `rec` from the LDS array `dist`.  freeb == nullptr: the array is
// in the record's format (get_state, before any finish pass); else its blocked cells hold +inf
// (after sssp_finish) and the rect's free bits decide.
__device__ __forceinline__ void rec_export(char *rec, const float *dist, int h, int w, int src_ok, const B128 *freeb, int t,
                                           int n)
{
    const int pw = (w + 2) | 1, cells = (h + 2) * pw;
    float *d = reinterpret_cast<float *>(rec + REC_HDR);
    if (!freeb) {
        const float4 *s4 = reinterpret_cast<const float4 *>(dist);  // (LDS array and record: 16-aligned)
        float4 *d4 = reinterpret_cast<float4 *>(d);
        for (int k = t; k < cells / 4; k += n) d4[k] = s4[k];
        for (int k = (cells & ~3) + t; k < cells; k += n) d[k] = dist[k];
    } else {
        for (int r = t / 128; r < h + 2; r += n / 128) {  // (row, column) walk: no division per cell
            const bool row_in = r >= 1 && r <= h;
            for (int c = t % 128; c < pw; c += 128) {
                const bool fr = row_in && c >= 1 && c <= w && b_test(freeb[r - 1], c - 1);
                d[r * pw + c] = fr ? dist[r * pw + c] : -INFINITY;
            }
        }
    }
    if (t == 0) *reinterpret_cast<int4 *>(rec) = make_int4(1, src_ok, h, w);
}
// byte offset (from distance array 0) of the distance phase's cell table when it lives in that
// array's unused tail (tail_cells: the table, 96 * 96 u16, fits after the room's cells)
__device__ __forceinline__ int tail_cells_off(int h, int w) { return ((h + 2) * sssp_pitch(w) * 4 + 15) & ~15; }

// G threads cover the window: words 0-1 of a row (columns 0..127): thread -> (row t / 128 + (G / 128) q,
// column t % 128), so every wave holds 64 consecutive columns of one row (one ballot per row word);
// word 2 (columns 128..133): thread -> (row 8 * wave + lane / 8 + (G / 8) u, column 128 + lane % 8).
template <int G>
struct OccLoad {
    static constexpr int NQ = 16384 / G, NU = 1024 / G;  // 128 rows x 128 columns, 128 rows x 8 columns
    uint8_t v[NQ], v2[NU];
};
template <int G>
__device__ __forceinline__ void cspace_load(OccLoad<G> &L, const uint8_t *__restrict__ occ, int H, int W, int i0, int j0,
                                            int h, int w, int t)
{
    // Unconditional buffer loads: a cell outside the map or the window gets offset 0xffffffff, which
    // the buffer's range check turns into 0 -- no exec-masked branch per load, so all of them are in
    // flight at once (bounds-checked pointer loads compiled to one branch + vmcnt(0) round trip each).
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)occ, (short)0, H * W, 0x00020000);
    const int lane = t & 63, wave = t >> 6;
    const int wh = h + 2 * RMAX, ww = w + 2 * RMAX;  // <= 126 x 134
    const int c = t & 127, r0 = t >> 7;
#pragma unroll
    for (int q = 0; q < OccLoad<G>::NQ; q++) {
        const int rr = r0 + (G / 128) * q, gi = i0 - RMAX + rr, gj = j0 - RMAX + c;
        const bool in = ((unsigned)rr < (unsigned)wh) & ((unsigned)c < (unsigned)ww) & ((unsigned)gi < (unsigned)H) &
                        ((unsigned)gj < (unsigned)W);
        L.v[q] = __builtin_amdgcn_raw_buffer_load_b8(rs, in ? gi * W + gj : -1, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < OccLoad<G>::NU; u++) {
        const int rr = 8 * wave + (lane >> 3) + (G / 8) * u, cc = 128 + (lane & 7), gi = i0 - RMAX + rr, gj = j0 - RMAX + cc;
        const bool in = ((unsigned)rr < (unsigned)wh) & ((unsigned)cc < (unsigned)ww) & ((unsigned)gi < (unsigned)H) &
                        ((unsigned)gj < (unsigned)W);
        L.v2[u] = __builtin_amdgcn_raw_buffer_load_b8(rs, in ? gi * W + gj : -1, 0, 0);
    }
}

// Byte loads + ballots straight into S.win, CH rows of loads in flight at a time (the sweep track's
// fallback when the dword variant's alignment bounds fail): a few registers instead of NQ + NU.
template <int G>
__device__ __forceinline__ void win_from_bytes(SsspScratch &S, const uint8_t *__restrict__ occ, int H, int W, int i0,
                                               int j0, int h, int w, int t)
{
    constexpr int NQ = 16384 / G, NU = 1024 / G, CH = 8;
    static_assert(NQ % CH == 0, "whole chunks");
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)occ, (short)0, H * W, 0x00020000);
    const int lane = t & 63, wave = t >> 6;
    const int wh = h + 2 * RMAX, ww = w + 2 * RMAX;
    const int c = t & 127, r0 = t >> 7;
#pragma unroll 1
    for (int q0 = 0; q0 < NQ; q0 += CH) {
        uint32_t v[CH];
#pragma unroll
        for (int k = 0; k < CH; k++) {
            const int rr = r0 + (G / 128) * (q0 + k), gi = i0 - RMAX + rr, gj = j0 - RMAX + c;
            const bool in = ((unsigned)rr < (unsigned)wh) & ((unsigned)c < (unsigned)ww) & ((unsigned)gi < (unsigned)H) &
                            ((unsigned)gj < (unsigned)W);
            v[k] = __builtin_amdgcn_raw_buffer_load_b8(rs, in ? gi * W + gj : -1, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < CH; k++) {
            const int rr = r0 + (G / 128) * (q0 + k);
            const uint64_t m = __ballot(v[k] != 0);
            if (lane == 0 && rr < wh) S.win[rr][wave & 1] = m;
        }
    }
    uint32_t v2[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int rr = 8 * wave + (lane >> 3) + (G / 8) * u, cc = 128 + (lane & 7), gi = i0 - RMAX + rr, gj = j0 - RMAX + cc;
        const bool in = ((unsigned)rr < (unsigned)wh) & ((unsigned)cc < (unsigned)ww) & ((unsigned)gi < (unsigned)H) &
                        ((unsigned)gj < (unsigned)W);
        v2[u] = __builtin_amdgcn_raw_buffer_load_b8(rs, in ? gi * W + gj : -1, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int rb = 8 * wave + (G / 8) * u;
        const uint64_t m = __ballot(v2[u] != 0);
        if (lane < 8 && rb + lane < wh) S.win[rb + lane][2] = (m >> (8 * lane)) & 0xffu;
    }
}

// Dword variant (the sweep track, G threads, rows 4-byte aligned in a map whose window columns lie
// inside it): each load covers 4 window columns from the aligned column a0 = (j0 - RMAX) & ~3, so the
// window rows land shifted by sub = (j0 - RMAX) - a0 bits, which the dilation's funnel shifts absorb.
// 128 rows x 32 dwords (columns 0..127) as 2 rows per wave load, + 128 rows x 4 dwords (128..143).
template <int G>
struct OccLoad4 {
    static constexpr int NQ = 4096 / G, NU = 512 / G;
    uint32_t v[NQ], v2[NU];
    int sub;
};
__host__ __device__ __forceinline__ bool occ4_ok(int H, int W, int j0)
{
    const int a0 = (j0 - RMAX) & ~3;
    return (W & 3) == 0 && j0 - RMAX >= 0 && a0 + 144 <= W;
}
template <int G>
__device__ __forceinline__ void cspace_load4(OccLoad4<G> &L, const uint8_t *__restrict__ occ, int H, int W, int i0, int j0,
                                             int h, int t)
{
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)occ, (short)0, H * W, 0x00020000);
    const int lane = t & 63, wave = t >> 6;
    const int wh = h + 2 * RMAX, a0 = (j0 - RMAX) & ~3;
    L.sub = (j0 - RMAX) - a0;
#pragma unroll
    for (int q = 0; q < OccLoad4<G>::NQ; q++) {
        const int rr = 2 * (wave + (G / 64) * q) + (lane >> 5), gi = i0 - RMAX + rr;
        const bool in = ((unsigned)rr < (unsigned)wh) & ((unsigned)gi < (unsigned)H);
        L.v[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, in ? gi * W + a0 + 4 * (lane & 31) : -1, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < OccLoad4<G>::NU; u++) {
        const int k = t + G * u, rr = k >> 2, gi = i0 - RMAX + rr;
        const bool in = ((unsigned)rr < (unsigned)wh) & ((unsigned)gi < (unsigned)H);
        L.v2[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, in ? gi * W + a0 + 128 + 4 * (k & 3) : -1, 0, 0);
    }
}
// bit b of the result = (byte b of x != 0), b = 0..3
__device__ __forceinline__ unsigned nib4(unsigned x)
{
    x |= x >> 4;
    x |= x >> 2;
    x |= x >> 1;  // bit 8b = OR of byte b's bits
    return ((x & 0x01010101u) * 0x01020408u) >> 24;
}
template <int G>
__device__ __forceinline__ void win_from_dwords(SsspScratch &S, const OccLoad4<G> &L, int whM, int t)
{
    const int lane = t & 63, wave = t >> 6;
    uint32_t *win32 = reinterpret_cast<uint32_t *>(&S.win[0][0]);
#pragma unroll
    for (int q = 0; q < OccLoad4<G>::NQ; q++) {
        // the 8 nibbles of lanes 8j .. 8j + 7 are word j of a row: OR them into lane 8j + 7
        unsigned x = nib4(L.v[q]) << (4 * (lane & 7));
        x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
        x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
        x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
        const int rr = 2 * (wave + (G / 64) * q) + (lane >> 5);
        if ((lane & 7) == 7 && rr < whM) win32[rr * 6 + ((lane >> 3) & 3)] = x;
    }
#pragma unroll
    for (int u = 0; u < OccLoad4<G>::NU; u++) {
        const int k = t + G * u, rr = k >> 2;
        unsigned x = nib4(L.v2[u]) << (4 * (k & 3));
        x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, true);
        x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xf, 0xf, true);
        if ((k & 3) == 3 && rr < whM) win32[rr * 6 + 4] = x;
    }
}

// OR of x over the 16 lanes of its DPP row (quad swaps, then half-row and row mirrors)
__device__ __forceinline__ unsigned row16_or(unsigned x)
{
    x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xf, 0xf, false);  // row_half_mirror
    x |= (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xf, 0xf, false);  // row_mirror
    return x;
}

// S.win rows (RMAX-window coordinates) -> S.freeb: 1 - max(1 - room_mask, binary_dilation(occ, disk(r)))
// inside the room rect (envs.py:2453).  No LDS staging, no atomics: window words come straight from
// the loaded registers by ballots; each 16-lane DPP row computes one output row, lane = disk row dy.
// Group g (g.n == G threads) -- the whole workgroup, or the sweep group while the render group works.
// With dist (the get_state sweep track), the 16 lanes that compute a row's free bits also write
// that row of every distance array (free +inf, blocked / border -inf; sssp_init_sources then sets
// the snapped sources to 0): no separate init pass over the arrays.
// The occupancy window comes from registers loaded earlier (L4: dword loads; L: byte loads) or, with
// neither, is loaded here in chunks (win_from_bytes on occ / H / W / i0 / j0).
template <int G>
__device__ __forceinline__ void build_cspace(SsspScratch &S, const OccLoad<G> *L, int h, int w, int r, const Group &g,
                                             float *dist = nullptr, int nsrc = 0, const OccLoad4<G> *L4 = nullptr,
                                             const uint8_t *occ = nullptr, int H = 0, int W = 0, int i0 = 0, int j0 = 0)
{
    const int t = g.t, lane = t & 63, wave = t >> 6;
    const int whM = h + 2 * RMAX, wwM = w + 2 * RMAX;
    const int sub = L4 ? L4->sub : 0;  // window bit k = column k - sub (dword loads)
    if (L4) {
        win_from_dwords<G>(S, *L4, whM, t);
    } else if (!L) {
        win_from_bytes<G>(S, occ, H, W, i0, j0, h, w, t);
    } else {
        const int c = t & 127, r0 = t >> 7;
#pragma unroll
        for (int q = 0; q < OccLoad<G>::NQ; q++) {
            const int rr = r0 + (G / 128) * q;
            const uint64_t m = __ballot(L->v[q] != 0);  // 0 outside the window (cspace_load)
            if (lane == 0 && rr < whM) S.win[rr][wave & 1] = m;
#ifdef SIMAPS_PHASE_STAMPS
            if (q == 0 && t == 0) STAMP_NB(46);
#endif
        }
#ifdef SIMAPS_PHASE_STAMPS
        if (t == 0) STAMP_NB(47);
#endif
#pragma unroll
        for (int u = 0; u < OccLoad<G>::NU; u++) {
            const int rb = 8 * wave + (G / 8) * u, rr = rb + (lane >> 3), cc = 128 + (lane & 7);
            const uint64_t m = __ballot(L->v2[u] != 0);
            if (lane < 8 && rb + lane < whM) S.win[rb + lane][2] = (m >> (8 * lane)) & 0xffu;
        }
    }
    g.sync();
    if (t == 0) STAMP_NB(15);
    const B128 fm = b_mask(w);
    const int ln = t & 63;
    const int dy = (t & 15) - r;
    int hw = -1;  // disk(r) half-width of row dy (skimage disk: dx^2 + dy^2 <= r^2)
    if (dy <= r)
        while ((hw + 1) * (hw + 1) + dy * dy <= r * r) hw++;
    const int pw = sssp_pitch(w);
    if (t == 0) STAMP_CLK(52);
    if (dist) {  // border rows 0 and h + 1
        for (int k = t; k < pw; k += G)
            for (int s = 0; s < nsrc; s++) {
                dist[s * DIST_FLOATS + k] = -INFINITY;
                dist[s * DIST_FLOATS + (h + 1) * pw + k] = -INFINITY;
            }
    }
    if (t == 0) STAMP_CLK(53);
    // Each wave owns a block of R = ceil(h / waves) consecutive output rows r0 .. r0 + R - 1 and
    // builds the window rows they need itself, once, so no group barrier separates the two steps
    // (neighbouring waves rewrite a few shared table rows with identical values):
    // (1) one lane per window row r0 + RMAX - r + lane (lane < R + 2r): its horizontal dilations by
    //     +-j (j = 0 .. r) over the rect columns, T_j = T_{j-1} | (row >> (RMAX + j)) |
    //     (row >> (RMAX - j)) (128-bit windows of the 192-bit row, compile-time shifts);
    // (2) 4 output rows per step, 16 lanes per row, lane = disk row dy: one table read, then a DPP
    //     OR over the lanes.
    constexpr int NW = G / 64;
    static_assert((MAX_ROWS + NW - 1) / NW + 2 * RMAX <= 64, "one table lane per window row");
    const int R = (h + NW - 1) / NW;
    const int r0 = wave * R;
    {
        if (r0 < h) {
            const int wr = r0 + RMAX - r + ln;
            if (ln < R + 2 * r && wr < whM) {
                const uint64_t x0 = S.win[wr][0], x1 = S.win[wr][1], x2 = S.win[wr][2];
                const uint32_t d[5] = {(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32), (uint32_t)x2};
                // bits s_ .. s_ + 127 of the row (s_ <= 2 RMAX < 32): one funnel shift per dword
                auto win4 = [&](int s_, int k) { return __builtin_amdgcn_alignbit(d[k + 1], d[k], s_ + sub); };
                uint32_t T[4];
#pragma unroll
                for (int k = 0; k < 4; k++) T[k] = win4(RMAX, k);
                S.dtab[0][wr] = B128{T[0] | ((uint64_t)T[1] << 32), T[2] | ((uint64_t)T[3] << 32)};
#pragma unroll
                for (int j = 1; j <= RMAX; j++) {
                    if (j <= r) {
#pragma unroll
                        for (int k = 0; k < 4; k++) T[k] |= win4(RMAX + j, k) | win4(RMAX - j, k);
                        S.dtab[j][wr] = B128{T[0] | ((uint64_t)T[1] << 32), T[2] | ((uint64_t)T[3] << 32)};
                    }
                }
            }
            // the wave's own LDS writes precede its reads (in-order LDS); keep the compiler in order
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    for (int sub = 0; sub < R; sub += 4) {  // uniform: every lane takes part in the DPP ORs
        const int row = r0 + sub + (ln >> 4);
        const bool own = sub + (ln >> 4) < R && row < h;
        B128 acc = {0, 0};
        if (own && hw >= 0) acc = S.dtab[hw][row + RMAX + dy];
#ifdef SIMAPS_PHASE_STAMPS
        if (t == 0 && sub == 0) { asm volatile("" ::"v"(acc.lo), "v"(acc.hi)); STAMP_CLK(54); }
#endif
        const unsigned a0 = row16_or((unsigned)acc.lo), a1 = row16_or((unsigned)(acc.lo >> 32));
        const unsigned a2 = row16_or((unsigned)acc.hi), a3 = row16_or((unsigned)(acc.hi >> 32));
#ifdef SIMAPS_PHASE_STAMPS
        if (t == 0 && sub == 0) { asm volatile("" ::"v"(a0), "v"(a3)); STAMP_CLK(55); }
#endif
        const uint64_t lo = ((uint64_t)a1 << 32) | a0, hi = ((uint64_t)a3 << 32) | a2;
        const B128 fr = {~lo & fm.lo, ~hi & fm.hi};
        if ((t & 15) == 0 && own) S.freeb[row] = fr;
        if (dist && own) {  // array column c = rect column c - 1 (fr << 1: column 0 and c > w blocked)
            const uint64_t f1lo = fr.lo << 1, f1hi = (fr.hi << 1) | (fr.lo >> 63);
            const uint32_t part[4] = {(uint32_t)f1lo, (uint32_t)(f1lo >> 32), (uint32_t)f1hi, (uint32_t)(f1hi >> 32)};
            float *drow = dist + (row + 1) * pw;
            const int l16 = t & 15;
            if (pw == 95 && nsrc == 2) {  // BASELINE rooms, two sources: c = 95 is the next row's border
#pragma unroll
                for (int i = 0; i < 6; i++) {
                    const int c = l16 + 16 * i;
                    const float v = ((part[i >> 1] >> (l16 + 16 * (i & 1))) & 1u) ? INFINITY : -INFINITY;
                    drow[c] = v;
                    drow[DIST_FLOATS + c] = v;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; i++) {  // c = l16 + 16 i < pw <= 123
                    const int c = l16 + 16 * i;
                    if (16 * i < pw) {
                        const float v = ((part[i >> 1] >> (l16 + 16 * (i & 1))) & 1u) ? INFINITY : -INFINITY;
                        if (c < pw)
                            for (int s = 0; s < nsrc; s++) drow[s * DIST_FLOATS + c] = v;
                    }
                }
            }
        }
#ifdef SIMAPS_PHASE_STAMPS
        if (t == 0) STAMP_CLK(sub == 0 ? 56 : 57);
#endif
    }
    if (t == 0) STAMP_CLK(58);
    g.sync();
    if (t == 0) STAMP_CLK(59);
}

// ------------------------------------------------------------------------------------------------
// Phase: snap the query pixels to the closest free cell (scipy EDT feature transform at q)
// ------------------------------------------------------------------------------------------------
template <class SH, class SC>  // Shared (get_state / sp_distance) or PathHdr (path kernels) / LookupHdr;
                               // SsspScratch or any struct with the rect's freeb rows
__device__ __forceinline__ void snap_sources(SH &sh, SC &S, int nsrc, const Group &g)
{
    const int tid = g.t;
    const int h = sh.h, w = sh.w, i0 = sh.i0, j0 = sh.j0;
    // fast path (the common case): a free query pixel is its own nearest free cell (EDT distance 0)
    if (tid < nsrc) {
        const int qr = sh.src_q[tid][0] - i0, qc = sh.src_q[tid][1] - j0;
        const bool fr = qr >= 0 && qr < h && qc >= 0 && qc < w && b_test(S.freeb[qr], qc);
        sh.src_ok[tid] = fr;
        if (fr) {
            sh.src_s[tid][0] = sh.src_q[tid][0];
            sh.src_s[tid][1] = sh.src_q[tid][1];
        }
    }
    g.sync();
    if (tid == 0) STAMP_NB(76);
    bool slow = false;
    for (int s = 0; s < nsrc; s++) slow |= !sh.src_ok[s];
    if (!slow) return;
    // scipy's feature transform at the query (pass 1 along axis 0: per column the nearest free row,
    // ties low; pass 2 along axis 1 at the query row: the lower envelope of (row - qi)^2 + (col - qj)^2,
    // which yields the minimising column, the lowest one on a tie -- a member is dropped only if its
    // interval is strictly empty and the query scan stops at the first member the next one does not
    // strictly beat; checked against scipy's serial envelope code on 2 x 10^5 random cases, 1.2 x 10^4
    // of them with ties).  One wave per source, lane l owning rect columns l and l + 64: rows are
    // scanned outward from the query row (qr - d before qr + d: ties low), every column at once,
    // until no column still searching can reach the best (d^2 + dc^2, column) key found so far.
    const int lane = tid & 63, wv = tid >> 6;
    if (wv < nsrc && !sh.src_ok[wv]) {
        const int s = wv;
        const int qi = __builtin_amdgcn_readfirstlane(sh.src_q[s][0]);
        const int qj = __builtin_amdgcn_readfirstlane(sh.src_q[s][1]);
        const int qr = qi - i0, qc = qj - j0;
        int rowd[2] = {-1, -1}, row[2] = {0, 0};  // per column: the nearest free row's distance / row
        // (d^2 + dc^2) << 7 | column: the lexicographic minimum, 64-bit (the query is clamped to the
        // grid only, so d and dc reach the grid size)
        long long best = 0x7fffffffffffffffll;
        const int dmax = max(abs(qr), abs(qr - (h - 1)));  // the farthest rect row from the query row
        for (int d = 0; d <= dmax; d++) {
            const long long dd = (long long)d * d;
            if (dd << 7 > best) break;  // no column still searching can reach the best key
            const int ra = qr - d, rb = qr + d;
            const bool va = ra >= 0 && ra < h, vb = d > 0 && rb >= 0 && rb < h;
            if (!va && !vb && ra < 0 && rb >= h) break;  // every row visited
            const B128 fa = va ? S.freeb[ra] : B128{0ull, 0ull};
            const B128 fb = vb ? S.freeb[rb] : B128{0ull, 0ull};
            for (int k = 0; k < 2; k++) {
                const int c = lane + 64 * k;
                if (c < w && rowd[k] < 0) {
                    if (b_test(fa, c)) { rowd[k] = d; row[k] = ra; }
                    else if (b_test(fb, c)) { rowd[k] = d; row[k] = rb; }
                    if (rowd[k] >= 0) {
                        const long long key = (((long long)d * d + (long long)(c - qc) * (c - qc)) << 7) | c;
                        best = min(best, key);
                    }
                }
            }
            for (int off = 32; off > 0; off >>= 1) best = min(best, __shfl_xor(best, off));
        }
        if (best != 0x7fffffffffffffffll) {  // (no free cell at all: src_ok stays 0)
            const int c = (int)(best & 127);
            const int owner = c & 63, k = c >> 6;
            const int r = __shfl(k ? row[1] : row[0], owner);
            if (lane == 0) {
                sh.src_s[s][0] = i0 + r;
                sh.src_s[s][1] = j0 + c;
                sh.src_ok[s] = 1;
            }
        }
    }
    g.sync();
}

// snap_sources' slow path for one query pixel (qi, qj) on one wave (wave-uniform, anywhere in the grid;
// occupancy_map_kernel).  The same algorithm, kept apart so that the kernels calling snap_sources keep
// their code bit for bit (tools/isa_digest.py: folding snap_sources onto it moved the get_state
// kernel's register allocation).  scipy's
// feature transform at the query (pass 1 along axis 0: per column the nearest free row, ties low;
// pass 2 along axis 1 at the query row: the lower envelope of (row - qi)^2 + (col - qj)^2, which yields
// the minimising column, the lowest one on a tie -- a member is dropped only if its interval is
// strictly empty and the query scan stops at the first member the next one does not strictly beat;
// checked against scipy's serial envelope code on 2 x 10^5 random cases, 1.2 x 10^4 of them with
// ties).  Lane l owns rect columns l and l + 64: rows are scanned outward from the query row (qr - d
// before qr + d: ties low), every column at once, until no column still searching can reach the best
// (d^2 + dc^2, column) key found so far.  found(si, sj) is called by every lane with the snapped cell,
// not at all if the rect has no free cell.
template <class F>
__device__ __forceinline__ void snap_wave(const B128 *freeb, int h, int w, int i0, int j0, int qi, int qj, F &&found)
{
    const int lane = threadIdx.x & 63;
    const int qr = qi - i0, qc = qj - j0;
    int rowd[2] = {-1, -1}, row[2] = {0, 0};  // per column: the nearest free row's distance / row
    // (d^2 + dc^2) << 7 | column: the lexicographic minimum, 64-bit (the query is clamped to the
    // grid only, so d and dc reach the grid size)
    long long best = 0x7fffffffffffffffll;
    const int dmax = max(abs(qr), abs(qr - (h - 1)));  // the farthest rect row from the query row
    for (int d = 0; d <= dmax; d++) {
        const long long dd = (long long)d * d;
        if (dd << 7 > best) break;  // no column still searching can reach the best key
        const int ra = qr - d, rb = qr + d;
        const bool va = ra >= 0 && ra < h, vb = d > 0 && rb >= 0 && rb < h;
        if (!va && !vb && ra < 0 && rb >= h) break;  // every row visited
        const B128 fa = va ? freeb[ra] : B128{0ull, 0ull};
        const B128 fb = vb ? freeb[rb] : B128{0ull, 0ull};
        for (int k = 0; k < 2; k++) {
            const int c = lane + 64 * k;
            if (c < w && rowd[k] < 0) {
                if (b_test(fa, c)) { rowd[k] = d; row[k] = ra; }
                else if (b_test(fb, c)) { rowd[k] = d; row[k] = rb; }
                if (rowd[k] >= 0) {
                    const long long key = (((long long)d * d + (long long)(c - qc) * (c - qc)) << 7) | c;
                    best = min(best, key);
                }
            }
        }
        for (int off = 32; off > 0; off >>= 1) best = min(best, __shfl_xor(best, off));
    }
    if (best != 0x7fffffffffffffffll) {  // (no free cell at all: not found)
        const int c = (int)(best & 127);
        const int owner = c & 63, k = c >> 6;
        const int r = __shfl(k ? row[1] : row[0], owner);
        found(i0 + r, j0 + c);
    }
}

// ------------------------------------------------------------------------------------------------
// Phase: single-source shortest paths for nsrc sources over the free cells of the rect
// ------------------------------------------------------------------------------------------------
// Directional sweeps.  Per source, four waves sweep the LDS-resident distance array concurrently:
// down / up (row by row, lanes own 2 columns each) and right / left (column by column, lanes own 2
// rows each).  A sweep step relaxes every cell of a line from the 3 cells of the previous line
// (straight + 2 diagonals); the previous line's new values stay in registers and reach the
// neighbouring lanes by DPP wave shifts, so a path that is monotone in the sweep direction is
// settled in ONE pass.  Rounds of 4 concurrent sweeps repeat until a round changes nothing.
// Every write is an LDS atomic min(current, fl(d_u + w)) for a real edge -- a valid relaxation
// that never raises a cell, even when another sweep improved it after this wave prefetched it --
// so rounds terminate, and a round without any candidate below the prefetched values (which are
// >= the current ones) proves the fixpoint: the unique float32 fixpoint = the reference SPFA's
// distances, bit for bit.
// Layout: dist[s] = (h + 2) x pitch float32 with a border, pitch = (w + 2) | 1 (odd: column-wise
// sweeps hit at most 2-way LDS bank conflicts).  Free cells start at +inf, blocked and border
// cells hold -inf: `candidate < cell` is false for them, so they are never written, and the value
// a lane passes on to the next line, |min(candidate, cell)|, is +inf for them (propagates nothing;
// the fabs is a free source modifier of the consumers).  No NaN anywhere, no free-bit tests.

// Rotations (no invalid source lanes, no `old` operand): lane 0 / lane 63 receive lane 63 / lane 0,
// which never own a cell (spans are <= 63 cells for 1 cell per lane, <= 120 for 2), so they carry
// +inf.
// (bound_ctrl set: a full-wave rotation has no invalid source lane, and it lets the compiler fold the
// move into its consumer -- v_add_f32_dpp with the |.| source modifier)
__device__ __forceinline__ float from_prev_lane(float v)  // lane i <- lane i-1
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x13c, 0xf, 0xf, true));  // wave_ror:1
}
__device__ __forceinline__ float from_next_lane(float v)  // lane i <- lane i+1
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x134, 0xf, 0xf, true));  // wave_rol:1
}


constexpr unsigned NINF_BITS = 0xff800000u;  // blocked / border cells

typedef __attribute__((address_space(3))) float lds_float;

// Unconditional ds_min_f32 of every lane, visible to the compiler.  (An `if (on) atomicMin` splits the
// step into exec-masked basic blocks no scheduling crosses; a masked inline-asm ds_min is invisible
// to the compiler's lgkmcnt bookkeeping, so each prefetch wait also drained the previous steps'
// atomics -- an LDS atomic round trip on every step of the chain.)  min(cell, m) with a real
// candidate m is a valid relaxation whether or not it improves the cell, and idle lanes write +inf
// to their own scratch cell, so no lane's write has to be masked.
__device__ __forceinline__ void lds_min(lds_float *p, float v)
{
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One sweep of one wave.  DIR: 0 down, 1 up (lines = rows), 2 right, 3 left (lines = columns);
// CPL: cells per lane across the line (1: span <= 63, 2: span <= 120); PWC: the pitch when known at
// compile time (0: runtime).  Returns true if a lane found an improvement.  Lines are prefetched P
// steps ahead into a ring of named registers.
// Every lane strides through memory the same way (one base per group of P steps, immediate offsets,
// no per-lane address arithmetic): lanes past the span alias the cells of active lanes and are made
// inert by per-lane constants instead of selects -- their edge weights are +inf (candidates +inf:
// the atomic min leaves the aliased cell alone and `candidate < cell` is false) and their passed-on
// value is minimum(., -inf) = -inf (|.| = +inf reaches the neighbouring lanes).
template <int DIR, int CPL, int PWC>
__device__ bool sweep_t(lds_float *__restrict__ D, int len, int span, int pw_rt)
{
    constexpr bool VERT = DIR < 2, FWD = (DIR & 1) == 0;
    constexpr int P = 4;
    const int pw = PWC ? PWC : pw_rt;
    const int lane = threadIdx.x & 63;
    const int sl = VERT ? pw : 1;             // address stride along the sweep (line to line)
    const int sa = VERT ? 1 : pw;             // across the line (cell 0 -> cell 1 of a lane)
    const int nact = (span + CPL - 1) / CPL;  // lanes owning a cell (>= 1)
    const bool act = lane < nact;
    const int own = act ? lane : lane & ((1 << (31 - __clz(nact))) - 1);
    lds_float *Dl = D + (1 + CPL * own) * sa;
    // line of step t: FWD 1 + t, else len - t.  Group base at step t0: lines t0 .. t0 + 2P - 1 at
    // non-negative offsets (ds offsets are unsigned)
    auto gbase = [&](int t0) { return FWD ? Dl + (1 + t0) * sl : Dl + (len - t0 - (2 * P - 1)) * sl; };
    auto goff = [&](int j) { return FWD ? j * sl : (2 * P - 1 - j) * sl; };
    float one = act ? 1.0f : INFINITY, s2 = act ? SQRT2F : INFINITY, X = act ? INFINITY : -INFINITY;
    asm volatile("" : "+v"(one), "+v"(s2), "+v"(X));  // VGPR operands (DPP-folded adds take no literal)
    const float NI = -INFINITY;
    lds_float *G = gbase(0);
    float A0 = G[goff(0)], A1 = CPL == 2 ? G[goff(0) + sa] : NI;
    float B0 = G[goff(1)], B1 = CPL == 2 ? G[goff(1) + sa] : NI;
    float C0 = G[goff(2)], C1 = CPL == 2 ? G[goff(2) + sa] : NI;
    float E0 = G[goff(3)], E1 = CPL == 2 ? G[goff(3) + sa] : NI;
    // p0 / p1: the previous line's values, -inf on blocked cells; consumers take |p| (a free source
    // modifier, also on the DPP-folded adds), so a blocked cell passes on +inf
    float p0 = INFINITY, p1 = INFINITY;       // the line before the first one: nothing
    uint64_t chg = 0;
#define SWEEP_STEP(R0, R1, J, LIVE)                                                                     \
    do {                                                                                                \
        float m0, m1 = INFINITY;                                                                        \
        if (CPL == 2) {                                                                                 \
            const float pm = from_prev_lane(p1), pp = from_next_lane(p0);                               \
            m0 = fminf(fminf(fabsf(p0) + one, fabsf(pm) + s2), fabsf(p1) + s2);                         \
            m1 = fminf(fminf(fabsf(p1) + one, fabsf(p0) + s2), fabsf(pp) + s2);                         \
        } else {                                                                                        \
            const float pm = from_prev_lane(p0), pp = from_next_lane(p0);                               \
            m0 = fminf(fminf(fabsf(p0) + one, fabsf(pm) + s2), fabsf(pp) + s2);                         \
        }                                                                                               \
        /* improvements as wave masks (v_cmp -> SGPRs, s_or): no per-lane flag arithmetic */            \
        const uint64_t u0 = (LIVE) ? __builtin_amdgcn_ballot_w64(m0 < R0) : 0;                          \
        const uint64_t u1 = CPL == 2 && (LIVE) ? __builtin_amdgcn_ballot_w64(m1 < R1) : 0;              \
        if (LIVE) { /* wave-uniform: steps past the last line write nothing */                          \
            SWEEP_WRITE(&G[goff(J)], m0, R0);                                                           \
            if (CPL == 2) SWEEP_WRITE(&G[goff(J) + sa], m1, R1);                                        \
        }                                                                                               \
        chg |= u0 | u1;                                                                                 \
        p0 = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m0, R0), X);                   \
        if (CPL == 2) p1 = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m1, R1), X);     \
        R0 = G[goff((J) + P)];                                                                          \
        if (CPL == 2) R1 = G[goff((J) + P) + sa];                                                       \
    } while (0)
#define SWEEP_WRITE(P_, V_, R_) lds_min((P_), (V_))
    int t = 0;
    for (; t + P <= len; t += P) {
        G = gbase(t);
        SWEEP_STEP(A0, A1, 0, true);
        SWEEP_STEP(B0, B1, 1, true);
        SWEEP_STEP(C0, C1, 2, true);
        SWEEP_STEP(E0, E1, 3, true);
    }
    if (t < len) {  // 1..3 remaining lines; steps past the end store nothing
        G = gbase(t);
        SWEEP_STEP(A0, A1, 0, t < len);
        SWEEP_STEP(B0, B1, 1, t + 1 < len);
        SWEEP_STEP(C0, C1, 2, t + 2 < len);
    }
#undef SWEEP_STEP
#undef SWEEP_WRITE
    return chg != 0;
}

// The same sweep as one inline-asm loop, for a compile-time pitch.  Measured on gfx950
// (tools/micro/issue.hip, one wave): every instruction costs the wave ~4.5 (VOP2 / SALU) to ~5.5
// (VOP3, DPP, v_cmp) cycles of issue, an SALU that consumes a v_cmp's SGPR result stalls ~16 more,
// ds_min_f32 ~9 alone / ~17 beside other LDS traffic -- dependent VALU latency is hidden.  So the
// step is minimised in instruction count, not in dependency depth:
//   - no per-step loop control: full groups of P = 4 steps, the first group and the tail peeled;
//   - changes are tracked in a VGPR, acc = min3(acc, m0 - R0, m1 - R1) (NaN from inf - inf is
//     ignored by v_min3), tested once at the end -- no v_cmp -> s_or per cell;
//   - exact lgkmcnt waits: step j waits only for line j's prefetch (issued P steps earlier);
//     the compiler's loop-merged bookkeeping drained the last steps' atomics instead.
// Every LDS operation, wait and register of the loop lives inside the asm, which drains
// (lgkmcnt(0)) before handing its registers back.  A DPP read of p0 / p1 follows their VALU write
// by >= 3 VALU instructions.
#define SWA_DSMIN(x) x
#define SWA_DSREAD(x) x
#define SWA_WAIT(W) "s_waitcnt lgkmcnt(" #W ")\n\t"
#define SWA_OFF(J) "((%[k0]+(" #J ")*%[kd])*%[sl4])"
#define SWA_ROR "wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
#define SWA_ROL "wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
// CPL 2: m0 = min3(|p0| + 1, prev-lane |p1| + s2, |p1| + s2), m1 = min3(|p1| + 1, |p0| + s2,
// next-lane |p0| + s2); p' = minimum3(m, R, X)
#define SWA_STEP2(RA0, RA1, J, W)                                                                  \
    "v_add_f32_e64 %[a], |%[p0]|, %[one]\n\t"                                                      \
    "v_add_f32_e64 %[d], |%[p1]|, %[one]\n\t"                                                      \
    "v_add_f32_e64 %[c], |%[p1]|, %[s2]\n\t"                                                       \
    "v_add_f32_e64 %[e], |%[p0]|, %[s2]\n\t"                                                       \
    "v_add_f32_dpp %[b], |%[p1]|, %[s2] " SWA_ROR "\n\t"                                           \
    "v_add_f32_dpp %[f], |%[p0]|, %[s2] " SWA_ROL "\n\t"                                           \
    "v_min3_f32 %[a], %[a], %[b], %[c]\n\t"                                                        \
    "v_min3_f32 %[d], %[d], %[e], %[f]\n\t"                                                        \
    SWA_DSMIN("ds_min_f32 %[va], %[a] offset:" SWA_OFF(J) "\n\t")                                  \
    SWA_DSMIN("ds_min_f32 %[va], %[d] offset:(" SWA_OFF(J) "+%[sa4])\n\t")                         \
    SWA_WAIT(W)                                                                                    \
    "v_minimum3_f32 %[p0], %[a], %[" #RA0 "], %[X]\n\t"                                            \
    "v_minimum3_f32 %[p1], %[d], %[" #RA1 "], %[X]\n\t"                                            \
    "v_sub_f32 %[b], %[a], %[" #RA0 "]\n\t"                                                        \
    "v_sub_f32 %[e], %[d], %[" #RA1 "]\n\t"                                                        \
    SWA_DSREAD("ds_read_b32 %[" #RA0 "], %[va] offset:" SWA_OFF(J + 4) "\n\t")                     \
    SWA_DSREAD("ds_read_b32 %[" #RA1 "], %[va] offset:(" SWA_OFF(J + 4) "+%[sa4])\n\t")            \
    "v_min3_f32 %[accg], %[accg], %[b], %[e]\n\t"
// CPL 1: m = min3(|p| + 1, prev-lane |p| + s2, next-lane |p| + s2)
#define SWA_STEP1(RA0, J, W)                                                                       \
    "v_add_f32_e64 %[a], |%[p0]|, %[one]\n\t"                                                      \
    "v_add_f32_dpp %[b], |%[p0]|, %[s2] " SWA_ROR "\n\t"                                           \
    "v_add_f32_dpp %[c], |%[p0]|, %[s2] " SWA_ROL "\n\t"                                           \
    "v_min3_f32 %[a], %[a], %[b], %[c]\n\t"                                                        \
    SWA_DSMIN("ds_min_f32 %[va], %[a] offset:" SWA_OFF(J) "\n\t")                                  \
    SWA_WAIT(W)                                                                                    \
    "v_minimum3_f32 %[p0], %[a], %[" #RA0 "], %[X]\n\t"                                            \
    "v_sub_f32 %[b], %[a], %[" #RA0 "]\n\t"                                                        \
    SWA_DSREAD("ds_read_b32 %[" #RA0 "], %[va] offset:" SWA_OFF(J + 4) "\n\t")                     \
    "v_min_f32 %[accg], %[b], %[accg]\n\t"
#define SWA_IFLEN(J) "s_cmp_le_i32 %[len], " #J "\n\t s_cbranch_scc1 3f\n\t"
#define SWA_IFREM(J) "s_cmp_le_i32 %[rem], " #J "\n\t s_cbranch_scc1 3f\n\t"
// After each full group: fold the group's change accumulator; a group that improved a cell records
// its step range [tg, tg + 3]; one that did not ends the sweep once it lies past the last dirty
// line (tg + 3 > tmax): every later line is clean, so the rest of the sweep would change nothing.
#define SWA_GROUP_END                                                                              \
    "v_cmp_gt_f32_e64 %[cm], 0, %[accg]\n\t"                                                       \
    "v_min_f32_e32 %[acc], %[accg], %[acc]\n\t"                                                    \
    "v_mov_b32_e32 %[accg], 0\n\t"                                                                 \
    "s_cmp_lg_u64 %[cm], 0\n\t"                                                                    \
    "s_cbranch_scc0 7f\n\t"                                                                        \
    "s_min_i32 %[imin], %[imin], %[tg]\n\t"                                                        \
    "s_add_i32 %[imax], %[tg], 3\n\t"                                                              \
    "s_branch 8f\n"                                                                                \
    "7:\n\t"                                                                                       \
    "s_cmp_gt_i32 %[tg], %[txm3]\n\t"                                                              \
    "s_cbranch_scc1 3f\n"                                                                          \
    "8:\n\t"                                                                                       \
    "s_add_i32 %[tg], %[tg], 4\n\t"
// lgkmcnt after the 2P prologue / steady-state reads: first group j -> ops issued after line j's read
#define SWA_BODY(STEP, R0_, R1_, R2_, R3_, W0, W1, W2, W3, WS)                                     \
    SWA_IFLEN(0) STEP(R0_, 0, W0) SWA_IFLEN(1) STEP(R1_, 1, W1) SWA_IFLEN(2) STEP(R2_, 2, W2)      \
    SWA_IFLEN(3) STEP(R3_, 3, W3)                                                                  \
    "v_add_u32_e32 %[va], %[gstep], %[va]\n\t"                                                     \
    SWA_GROUP_END                                                                                  \
    "s_cmp_eq_u32 %[ng], 0\n\t"                                                                    \
    "s_cbranch_scc1 2f\n"                                                                          \
    "1:\n\t"                                                                                       \
    STEP(R0_, 0, WS) STEP(R1_, 1, WS) STEP(R2_, 2, WS) STEP(R3_, 3, WS)                            \
    "v_add_u32_e32 %[va], %[gstep], %[va]\n\t"                                                     \
    SWA_GROUP_END                                                                                  \
    "s_sub_u32 %[ng], %[ng], 1\n\t"                                                                \
    "s_cmp_lg_u32 %[ng], 0\n\t"                                                                    \
    "s_cbranch_scc1 1b\n"                                                                          \
    "2:\n\t"                                                                                       \
    SWA_IFREM(0) STEP(R0_, 0, WS) SWA_IFREM(1) STEP(R1_, 1, WS) SWA_IFREM(2) STEP(R2_, 2, WS)      \
    "3:\n\t"                                                                                       \
    "v_cmp_gt_f32_e64 %[cm], 0, %[accg]\n\t"                                                       \
    "v_min_f32_e32 %[acc], %[accg], %[acc]\n\t"                                                    \
    "s_cmp_lg_u64 %[cm], 0\n\t"                                                                    \
    "s_cbranch_scc0 9f\n\t"                                                                        \
    "s_min_i32 %[imin], %[imin], %[tg]\n\t"                                                        \
    "s_add_i32 %[imax], %[tg], 3\n"                                                                \
    "9:\n\t"                                                                                       \
    "s_waitcnt lgkmcnt(0)\n\t"
#define SWA_S2(RA, J, W) SWA_STEP2(RA##0, RA##1, J, W)

// Result of one directional sweep: lanes that improved a cell anywhere (their lines, for the
// perpendicular directions) and the step range of the groups that improved one (for the opposite
// direction); imin > imax when nothing improved.
struct SweepOut {
    uint64_t lanes;
    int imin, imax;
    int steps;  // lines processed (diagnostics)
};

// Sweep steps t0 .. t1 - 1 (early exit past tmax) of a line space of len lines.
template <int DIR, int CPL, int PWC>
__device__ SweepOut sweep_asm(lds_float *__restrict__ D, int len, int span, int t0, int tmax, int t1)
{
    static_assert(PWC > 0, "compile-time pitch");
    constexpr bool VERT = DIR < 2, FWD = (DIR & 1) == 0;
    constexpr int P = 4;
    constexpr int SL = VERT ? PWC : 1, SA = VERT ? 1 : PWC;
    const int lane = threadIdx.x & 63;
    const int nact = (span + CPL - 1) / CPL;
    const bool act = lane < nact;
    const int own = act ? lane : lane & ((1 << (31 - __clz(nact))) - 1);
    lds_float *Dl = D + (1 + CPL * own) * SA;
    // group base at step t0; lines j = 0 .. 2P - 1 of a group at offset (k0 + j kd) * SL * 4 >= 0
    uint32_t va = (uint32_t)(uintptr_t)(FWD ? Dl + (1 + t0) * SL : Dl + (len - t0 - (2 * P - 1)) * SL);
    float one = act ? 1.0f : INFINITY, s2 = act ? SQRT2F : INFINITY, X = act ? INFINITY : -INFINITY;
    float p0 = INFINITY, p1 = INFINITY, acc = 0.0f, accg = 0.0f;
    float r00, r01, r10, r11, r20, r21, r30, r31, a, b, c, d, e, f;
    const int lenr = t1 - t0;                  // steps from t0 to the end
    int ng = lenr > P ? (lenr - P) / P : 0;    // steady-state groups after the first
    const int rem = lenr > P ? (lenr - P) % P : 0;
    const int txm3 = tmax - t0 - 3;
    int tg = 0, imin = 1 << 30, imax = -1;
    uint64_t cm;
    if constexpr (CPL == 2) {
        asm volatile(
            SWA_DSREAD("ds_read_b32 %[r00], %[va] offset:" SWA_OFF(0) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r01], %[va] offset:(" SWA_OFF(0) "+%[sa4])\n\t")
            SWA_DSREAD("ds_read_b32 %[r10], %[va] offset:" SWA_OFF(1) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r11], %[va] offset:(" SWA_OFF(1) "+%[sa4])\n\t")
            SWA_DSREAD("ds_read_b32 %[r20], %[va] offset:" SWA_OFF(2) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r21], %[va] offset:(" SWA_OFF(2) "+%[sa4])\n\t")
            SWA_DSREAD("ds_read_b32 %[r30], %[va] offset:" SWA_OFF(3) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r31], %[va] offset:(" SWA_OFF(3) "+%[sa4])\n\t")
            SWA_BODY(SWA_S2, r0, r1, r2, r3, 8, 10, 12, 14, 14)
            : [p0] "+v"(p0), [p1] "+v"(p1), [acc] "+v"(acc), [accg] "+v"(accg), [va] "+v"(va), [ng] "+s"(ng),
              [tg] "+s"(tg), [imin] "+s"(imin), [imax] "+s"(imax), [cm] "=&s"(cm), [r00] "=&v"(r00),
              [r01] "=&v"(r01), [r10] "=&v"(r10), [r11] "=&v"(r11), [r20] "=&v"(r20), [r21] "=&v"(r21),
              [r30] "=&v"(r30), [r31] "=&v"(r31), [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c), [d] "=&v"(d),
              [e] "=&v"(e), [f] "=&v"(f)
            : [one] "v"(one), [s2] "v"(s2), [X] "v"(X), [len] "s"(lenr), [rem] "s"(rem), [txm3] "s"(txm3),
              [k0] "i"(FWD ? 0 : 2 * P - 1), [kd] "i"(FWD ? 1 : -1), [sl4] "i"(SL * 4), [sa4] "i"(SA * 4),
              [gstep] "i"((FWD ? P : -P) * SL * 4)
            : "memory", "scc");
    } else {
        asm volatile(
            SWA_DSREAD("ds_read_b32 %[r00], %[va] offset:" SWA_OFF(0) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r10], %[va] offset:" SWA_OFF(1) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r20], %[va] offset:" SWA_OFF(2) "\n\t")
            SWA_DSREAD("ds_read_b32 %[r30], %[va] offset:" SWA_OFF(3) "\n\t")
            SWA_BODY(SWA_STEP1, r00, r10, r20, r30, 4, 5, 6, 7, 7)
            : [p0] "+v"(p0), [acc] "+v"(acc), [accg] "+v"(accg), [va] "+v"(va), [ng] "+s"(ng), [tg] "+s"(tg),
              [imin] "+s"(imin), [imax] "+s"(imax), [cm] "=&s"(cm), [r00] "=&v"(r00), [r10] "=&v"(r10),
              [r20] "=&v"(r20), [r30] "=&v"(r30), [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c)
            : [one] "v"(one), [s2] "v"(s2), [X] "v"(X), [len] "s"(lenr), [rem] "s"(rem), [txm3] "s"(txm3),
              [k0] "i"(FWD ? 0 : 2 * P - 1), [kd] "i"(FWD ? 1 : -1), [sl4] "i"(SL * 4),
              [gstep] "i"((FWD ? P : -P) * SL * 4)
            : "memory", "scc");
    }
    return SweepOut{__ballot(acc < 0.0f), t0 + imin, min(t0 + imax, t1 - 1), min(tg + 4, lenr)};
}
#undef SWA_S2
#undef SWA_BODY
#undef SWA_GROUP_END
#undef SWA_IFREM
#undef SWA_IFLEN
#undef SWA_STEP1
#undef SWA_STEP2
#undef SWA_ROL
#undef SWA_ROR
#undef SWA_OFF
#undef SWA_WAIT
#undef SWA_DSREAD
#undef SWA_DSMIN

// ---- dirty lines -------------------------------------------------------------------------------
// Each source keeps, per sweep direction, a 128-bit mask of the lines (bit L - 1 = line L) whose
// values changed since that direction last relaxed out of them.  Invariant: the current values of a
// clean line were relaxed (in that direction) into the next line.  A sweep snapshot-clears its mask,
// starts at its first dirty line and ends at the first group past its last dirty line that improves
// nothing; then it marks what it lowered: the lines of its improving steps for the opposite direction
// and the lines of its improving lanes for the two perpendicular ones (conservative supersets).
// Marks follow the sweep's own writes (its asm drains them) and a snapshot precedes the sweep's
// reads, so a decrease is either seen by a sweep or left marked for the next round.  A round in which
// nothing improves adds no marks and leaves every mask empty: the fixpoint.
__device__ __forceinline__ uint64_t spread2(uint32_t x)  // bit i -> bits 2i and 2i + 1
{
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v | (v << 1);
}
__device__ __forceinline__ uint64_t bits64(int a, int b)  // bits a .. b of a word, a <= b within [0, 63]
{
    return (b >= 63 ? ~0ull : ((1ull << (b + 1)) - 1)) & (~0ull << a);
}
__device__ __forceinline__ void mark_lines(uint64_t *m, uint64_t lo, uint64_t hi)
{
    if (lo) __hip_atomic_fetch_or(&m[0], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (hi) __hip_atomic_fetch_or(&m[1], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void mark_range(uint64_t *m, int a, int b)  // bits a .. b, 0 <= a <= b <= 127
{
    mark_lines(m, a <= 63 ? bits64(a, min(b, 63)) : 0ull, b >= 64 ? bits64(max(a, 64) - 64, b - 64) : 0ull);
}

// SSSP_CHECK: the rounds end with the fixpoint check below (sssp_check) instead of inline marks.
#ifdef SIMAPS_SSSP_CHECK
constexpr bool SSSP_CHECK = true;   // (A/B build: measured slower, HISTORY.md Appendix C)
#else
constexpr bool SSSP_CHECK = false;  // the product: inline marks + a confirming round
#endif

// One sweep of direction dir_in over source dm's array; true if it improved a cell.  With nparts > 1
// (compile-time pitch only) the sweep covers part `part` of the direction's steps: it relaxes out of
// the lines of steps [s0, s1) (their dirty bits are its own) and into the line of step s1, which the
// next part relaxes out of -- marked dirty for it when this part improved that line.
constexpr bool SSSP_INLINE_MARKS = !SSSP_CHECK;
__device__ __forceinline__ bool sweep(float *Dg, int h, int w, int pw, int dir_in, uint64_t (*dm)[2], int &steps,
                                      int part = 0, int nparts = 1, bool marks = SSSP_INLINE_MARKS)
{
    lds_float *D = (lds_float *)Dg;  // the distance arrays live in LDS: keep ds_* addressing
    // wave-uniform loop bounds: scalar loop control, no exec-mask merges at the back edge
    const int dir = __builtin_amdgcn_readfirstlane(dir_in);
    h = __builtin_amdgcn_readfirstlane(h);
    w = __builtin_amdgcn_readfirstlane(w);
    pw = __builtin_amdgcn_readfirstlane(pw);
    part = __builtin_amdgcn_readfirstlane(part);
    nparts = __builtin_amdgcn_readfirstlane(nparts);
    const bool vert = dir < 2, fwd = (dir & 1) == 0;
    const int len = vert ? h : w, span = vert ? w : h;
    const int lane = threadIdx.x & 63;
    // own steps [s0, s1) -> own dirty bits [b0, b1] (step t is line fwd ? t + 1 : len - t, bit line - 1)
    const int s0 = part * len / nparts, s1 = (part + 1) * len / nparts;
    const int b0 = fwd ? s0 : len - s1, b1 = fwd ? s1 - 1 : len - 1 - s0;
    uint64_t mlo = 0, mhi = 0;
    if (lane == 0) {  // snapshot-and-clear this direction's dirty lines (before any read of the array)
        if (nparts == 1) {
            mlo = __hip_atomic_exchange(&dm[dir][0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            mhi = __hip_atomic_exchange(&dm[dir][1], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            const uint64_t klo = b0 <= 63 ? bits64(b0, min(b1, 63)) : 0ull;
            const uint64_t khi = b1 >= 64 ? bits64(max(b0, 64) - 64, b1 - 64) : 0ull;
            if (klo) mlo = __hip_atomic_fetch_and(&dm[dir][0], ~klo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & klo;
            if (khi) mhi = __hip_atomic_fetch_and(&dm[dir][1], ~khi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & khi;
        }
    }
    mlo = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(mlo >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)mlo);
    mhi = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(mhi >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)mhi);
    if (!(mlo | mhi)) return false;
    const int blo = mlo ? __builtin_ctzll(mlo) : 64 + __builtin_ctzll(mhi);
    const int bhi = mhi ? 127 - __builtin_clzll(mhi) : 63 - __builtin_clzll(mlo);
    const int t0 = fwd ? blo : len - 1 - bhi, tmax = fwd ? bhi : len - 1 - blo;  // step t: line fwd ? t + 1 : len - t
    const int t1 = min(s1 + 1, len);
    if (pw == 95
    ) {  // every BASELINE room is 92 columns wide (pitch 95): the asm loop with immediate offsets
        SweepOut o;
        switch (dir) {
        case 0: o = sweep_asm<0, 2, 95>(D, h, w, t0, tmax, t1); break;
        case 1: o = sweep_asm<1, 2, 95>(D, h, w, t0, tmax, t1); break;
        case 2: o = h <= 63 ? sweep_asm<2, 1, 95>(D, w, h, t0, tmax, t1) : sweep_asm<2, 2, 95>(D, w, h, t0, tmax, t1); break;
        default: o = h <= 63 ? sweep_asm<3, 1, 95>(D, w, h, t0, tmax, t1) : sweep_asm<3, 2, 95>(D, w, h, t0, tmax, t1); break;
        }
        steps += o.steps;
        if (!o.lanes) return false;
        if (marks && lane == 0) {
            const int a = fwd ? o.imin : len - 1 - o.imax, b = fwd ? o.imax : len - 1 - o.imin;
            mark_range(dm[dir ^ 1], max(a, 0), min(b, 127));
            if (s1 < len && o.imax >= s1) {  // improved the next part's first line: its to relax out of
                const int bit = fwd ? s1 : len - 1 - s1;
                mark_range(dm[dir], bit, bit);
            }
            const int cpl = span <= 63 ? 1 : 2;
            const uint64_t lo = cpl == 1 ? o.lanes : spread2((uint32_t)o.lanes);
            const uint64_t hi = cpl == 1 ? 0ull : spread2((uint32_t)(o.lanes >> 32));
            const int p = vert ? 2 : 0;
            mark_lines(dm[p], lo, hi);
            mark_lines(dm[p + 1], lo, hi);
        }
        return true;
    }
    // runtime pitch: a full sweep; if it improved anything, every line of the others is marked
    bool chg;
    switch (dir) {
    case 0: chg = w <= 63 ? sweep_t<0, 1, 0>(D, h, w, pw) : sweep_t<0, 2, 0>(D, h, w, pw); break;
    case 1: chg = w <= 63 ? sweep_t<1, 1, 0>(D, h, w, pw) : sweep_t<1, 2, 0>(D, h, w, pw); break;
    case 2: chg = h <= 63 ? sweep_t<2, 1, 0>(D, w, h, pw) : sweep_t<2, 2, 0>(D, w, h, pw); break;
    default: chg = h <= 63 ? sweep_t<3, 1, 0>(D, w, h, pw) : sweep_t<3, 2, 0>(D, w, h, pw); break;
    }
    if (marks && chg && lane == 0)
        for (int d2 = 0; d2 < 4; d2++)
            if (d2 != dir) mark_range(dm[d2], 0, (d2 < 2 ? h : w) - 1);
    return chg;
}

// ---- the fixpoint check (round 4) -----------------------------------------------------------------
// After a round's sweeps (behind their barrier), one lane-parallel pass tests EVERY edge into every
// cell, fl(|d_u| + w) < d_v -- the relaxation a sweep step performs -- which is the fixpoint
// condition itself.  A cell with a violated edge marks every line such an edge can come out of
// (the rows above / below for the down / up sweeps, which relax the straight and both diagonal
// edges out of a row; the columns left / right for the right / left sweeps).  The next round
// sweeps only from those lines, and a round whose check finds no violated edge has reached the unique f32 fixpoint, so
// no confirmation round runs and a sweep leaves no marks behind (SSSP_CHECK; the inline marks
// are supersets: a lowered line is re-swept in the opposite direction whether or not anything
// there can improve).  Modelled first (tools/sssp_sched_sim.py: -29 % of the slowest sweep chain
// at an assumed ~1,500-cycle check) and built: bitwise, 3 rounds instead of 4 and -35 % line steps
// on the BASELINE config, but the check itself costs ~2.2 us per round in the kernel (~25 VALU
// per row on SIMDs shared with the render waves) plus a second barrier, so every config measured
// slower (HISTORY.md Appendix C).  Kept as the SIMAPS_SSSP_CHECK A/B build, not the product.
// Threads t of n (n = 64 * waves, this source's group): lane l owns columns 2l + 1, 2l + 2
// (w <= 126), wave q a block of rows; returns true (uniform per wave) if this wave found a violation.
__device__ __forceinline__ uint64_t spread_even(uint32_t x)  // bit i -> bit 2i
{
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}
__device__ __forceinline__ bool sssp_check(const float *Dg, int h, int w, int pw, uint64_t (*dm)[2], int t, int n)
{
    const lds_float *D = (const lds_float *)Dg;
    const int lane = t & 63, q = t >> 6, nw = n >> 6;
    h = __builtin_amdgcn_readfirstlane(h);
    w = __builtin_amdgcn_readfirstlane(w);
    pw = __builtin_amdgcn_readfirstlane(pw);
    // array rows [r0, r1), <= 32 of them (wave-uniform: scalar loop control)
    const int r0 = __builtin_amdgcn_readfirstlane(1 + q * h / nw), r1 = __builtin_amdgcn_readfirstlane(1 + (q + 1) * h / nw);
    const bool on0 = 2 * lane + 1 <= w, on1 = 2 * lane + 2 <= w;
    const int c0 = on0 ? 2 * lane + 1 : 1;  // (idle lanes alias lane 0's cells, masked below)
    const float s2 = SQRT2F, NI = -INFINITY;
    // A cell's best candidate over its 8 edges, min(|d_u| + w_uv), against its own value; a violated
    // cell (r, c) marks the down sweep at row r - 1, the up sweep at row r + 1, the right sweep at
    // column c - 1 and the left sweep at column c + 1 -- every line a violated edge into it can come
    // out of (a superset: a sweep that finds nothing there stops after one quiet group).  Per row, the
    // eight |x| + w of its four cells serve both as its vertical candidates for the rows above and
    // below and as its horizontal ones.
    struct RowC {
        float x0, x1;      // the row's two cells
        float v0, v1;      // what the row offers the cells (same columns) of the rows above / below
        float h0, h1;      // the best horizontal candidate of each of its two cells
    };
    auto row = [&](int rr) {
        const lds_float *p = D + rr * pw + c0 - 1;  // columns c0 - 1 .. c0 + 2
        const float a = p[0], b = p[1], c = p[2], d = p[3];
        const float a1 = fabsf(a) + 1.0f, b1 = fabsf(b) + 1.0f, c1 = fabsf(c) + 1.0f, d1 = fabsf(d) + 1.0f;
        const float as = fabsf(a) + s2, bs = fabsf(b) + s2, cs = fabsf(c) + s2, ds = fabsf(d) + s2;
        RowC o;
        o.x0 = on0 ? b : NI;  // -inf: never improvable
        o.x1 = on1 ? c : NI;
        o.v0 = __builtin_fminf(__builtin_fminf(as, b1), cs);
        o.v1 = __builtin_fminf(__builtin_fminf(bs, c1), ds);
        o.h0 = __builtin_fminf(a1, c1);
        o.h1 = __builtin_fminf(b1, d1);
        return o;
    };
    // rows of this wave in chunks of CK: the CK + 2 rows' loads are issued together (row indices
    // clamped into the array: a chunk past the wave's last row re-reads row r1, unused), then the
    // rows' candidates, then the CK checks -- one LDS round trip per chunk instead of one per row
    constexpr int CK = 8;
    uint32_t rbits = 0;      // bit (r - r0): row r holds a violated cell
    uint32_t cvb = 0;        // bit 0 / 1: this lane's column c0 / c0 + 1 holds a violated cell
    for (int rb = r0; rb < r1; rb += CK) {
        RowC R[CK + 2];
#pragma unroll
        for (int k = 0; k < CK + 2; k++) R[k] = row(min(rb - 1 + k, r1));
#pragma unroll
        for (int k = 1; k <= CK; k++) {
            const int r = rb - 1 + k;
            const bool e0 = __builtin_fminf(__builtin_fminf(R[k - 1].v0, R[k + 1].v0), R[k].h0) < R[k].x0;
            const bool e1 = __builtin_fminf(__builtin_fminf(R[k - 1].v1, R[k + 1].v1), R[k].h1) < R[k].x1;
            const uint32_t e = r < r1 ? (uint32_t)e0 | ((uint32_t)e1 << 1) : 0u;
            cvb |= e;
            rbits |= (e != 0u ? 1u : 0u) << (r - r0);
        }
    }
    const bool cv0 = cvb & 1u, cv1 = (cvb >> 1) & 1u;
    // rows: OR over the wave (DPP reductions), then the marks; columns: ballots
    uint32_t rb = rbits;
    rb |= __builtin_amdgcn_update_dpp(0, rb, 0x111, 0xf, 0xf, false);  // row_shr:1
    rb |= __builtin_amdgcn_update_dpp(0, rb, 0x112, 0xf, 0xf, false);  // row_shr:2
    rb |= __builtin_amdgcn_update_dpp(0, rb, 0x114, 0xf, 0xf, false);  // row_shr:4
    rb |= __builtin_amdgcn_update_dpp(0, rb, 0x118, 0xf, 0xf, false);  // row_shr:8
    rb |= __builtin_amdgcn_update_dpp(0, rb, 0x142, 0xa, 0xf, false);  // row_bcast:15
    rb |= __builtin_amdgcn_update_dpp(0, rb, 0x143, 0xc, 0xf, false);  // row_bcast:31
    const uint32_t rows = (uint32_t)__builtin_amdgcn_readlane((int)rb, 63);
    const uint64_t b0 = __ballot(cv0), b1 = __ballot(cv1);
    const bool any = (rows | b0 | b1) != 0;
    if (lane == 0 && any) {
        // violated row r (bit r - r0) -> down bit (r - 1) - 1 = r - 2, up bit (r + 1) - 1 = r
        const unsigned __int128 R = (unsigned __int128)rows << (r0 - 1);  // bit r - 1 (r >= 1)
        const unsigned __int128 Dn = R >> 1, Up = R << 1;
        // violated column c (lane l: 2l + 1 from b0, 2l + 2 from b1), bit c - 1 = 2l / 2l + 1 -> the
        // right sweep at column c - 1 (bit c - 2), the left sweep at column c + 1 (bit c)
        const unsigned __int128 Cc = ((unsigned __int128)spread_even((uint32_t)(b0 >> 32)) << 64 | spread_even((uint32_t)b0)) |
                                     (((unsigned __int128)spread_even((uint32_t)(b1 >> 32)) << 64 | spread_even((uint32_t)b1)) << 1);
        const unsigned __int128 Rt = Cc >> 1, Lt = Cc << 1;
        mark_lines(dm[0], (uint64_t)Dn, (uint64_t)(Dn >> 64));
        mark_lines(dm[1], (uint64_t)Up, (uint64_t)(Up >> 64));
        mark_lines(dm[2], (uint64_t)Rt, (uint64_t)(Rt >> 64));
        mark_lines(dm[3], (uint64_t)Lt, (uint64_t)(Lt >> 64));
    }
    return any;
}

// group g: free cells +inf, blocked / border -inf, sources 0 (one pass over the rect rows)
__device__ __forceinline__ void sssp_init(Shared &sh, const SsspScratch &S, float *dist, int nsrc, const Group &g)
{
    const int tid = g.t;
    const int h = sh.h, w = sh.w, pw = sssp_pitch(w);
    const float NI = -INFINITY;
    int sidx[2];  // flat index of each (snapped, free) source, -1 if none
    for (int s = 0; s < 2; s++)
        sidx[s] = (s < nsrc && sh.src_ok[s]) ? (sh.src_s[s][0] - sh.i0 + 1) * pw + (sh.src_s[s][1] - sh.j0 + 1) : -1;
    // (row, column) walk instead of k / pitch: integer division by a runtime value costs ~40 ops
    for (int rr = tid >> 7; rr < h + 2; rr += g.n >> 7) {
        const B128 fb = (rr >= 1 && rr <= h) ? S.freeb[rr - 1] : B128{0, 0};
        for (int c = tid & 127; c < pw; c += 128) {
            const int k = rr * pw + c;
            const float v = (c >= 1 && c <= w && b_test(fb, c - 1)) ? INFINITY : NI;
            for (int s = 0; s < nsrc; s++) dist[s * DIST_FLOATS + k] = k == sidx[s] ? 0.0f : v;
        }
    }
    if (tid < 6) (&sh.changed[0][0])[tid] = 0;
    if (tid == 6) sh.rounds = 0;
    if (tid < 8) {  // every line of every direction is dirty
        const int s = tid >> 2, d2 = tid & 3, n = d2 < 2 ? h : w;
        sh.dirty[s][d2][0] = n >= 64 ? ~0ull : (1ull << n) - 1;
        sh.dirty[s][d2][1] = n <= 64 ? 0ull : (n >= 128 ? ~0ull : (1ull << (n - 64)) - 1);
    }
    g.sync();
}

// group g, after build_cspace(dist) and snap_sources: the snapped (free) sources start at 0
__device__ __forceinline__ void sssp_init_sources(Shared &sh, float *dist, int nsrc, const Group &g)
{
    const int t = g.t, pw = sssp_pitch(sh.w);
    if (t < nsrc && sh.src_ok[t])
        dist[t * DIST_FLOATS + (sh.src_s[t][0] - sh.i0 + 1) * pw + (sh.src_s[t][1] - sh.j0 + 1)] = 0.0f;
    if (t < 6) (&sh.changed[0][0])[t] = 0;
    if (t == 6) sh.rounds = 0;
    if (t >= 64 && t < 64 + 16) {  // only the source's row / column is dirty (all else is +-inf)
        const int q = t - 64, s = q >> 3, d2 = (q >> 1) & 3, word = q & 1;
        const int bit = s < nsrc && sh.src_ok[s] ? (d2 < 2 ? sh.src_s[s][0] - sh.i0 : sh.src_s[s][1] - sh.j0) : -1;
        sh.dirty[s][d2][word] = bit >= 0 && (bit >> 6) == word ? 1ull << (bit & 63) : 0ull;
    }
    g.sync();
}

// the sweep group (waves 0 .. 4*nsrc-1): rounds of concurrent sweeps until one changes nothing
// the sweep waves (waves 0 .. 4*nsrc-1, four per source): rounds of concurrent sweeps until one
// changes nothing.  Each source runs its own rounds (its own 4-wave barrier and change flags): the
// two distance arrays are independent, so neither waits for the other's longest sweep.
__device__ __forceinline__ void sssp_rounds(Shared &sh, float *dist, int nsrc, const Group &)
{
    const int tid = threadIdx.x, wave = tid >> 6;
    const int h = sh.h, w = sh.w, pw = sssp_pitch(w);
    const int max_rounds = h * w + 16;  // a converged round changes nothing; the cap guards a bug
    const int s = wave >> 2;
    const Group gs{tid & 255, 256, sh.bar[2 + s], 4};
    int *changed = sh.changed[s];
    {   // issue priority over the render waves (which have slack), the longer sweeps first (VALU
        // arbitration is priority, then age)
        const int dir = (wave + 2 * s) & 3;
        if ((dir >= 2) == (w >= h)) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(2);
    }
    int steps = 0;  // lines this wave processed (diagnostics)
    for (int round = 0;; round++) {
        if ((tid & 255) == 0) changed[(round + 1) % 3] = 0;
#ifdef SIMAPS_PHASE_STAMPS
        if (tid == 0 && round < 4) STAMP_NB(18 + round);
        if (round == 0) STAMP_NB(32 + wave);
        if (round == 0 && wave == 0) STAMP_CLK(44);
#endif
        // waves go to SIMD (wave % 4): source 1's directions are rotated by 2 so that every SIMD
        // hosts one row sweep and one column sweep (the long ones would otherwise share two SIMDs)
        if (sh.src_ok[s] && sweep(dist + s * DIST_FLOATS, h, w, pw, (wave + 2 * s) & 3, sh.dirty[s], steps) && (tid & 63) == 0 &&
            !SSSP_CHECK)
            changed[round % 3] = 1;
#ifdef SIMAPS_PHASE_STAMPS
        if (round == 0 && wave == 0) STAMP_NB(22);
        if (round == 0 && wave == 2) STAMP_NB(23);
        if (round == 0) STAMP_NB(24 + wave);
        if (round == 0 && wave == 0) STAMP_CLK(45);
#endif
        gs.sync();
        if (SSSP_CHECK) {  // every edge; the violated ones mark the next round's lines
#ifdef SIMAPS_PHASE_STAMPS
            if (tid == 0 && round == 0) STAMP_NB(56);
#endif
            if (sh.src_ok[s] && sssp_check(dist + s * DIST_FLOATS, h, w, pw, sh.dirty[s], tid & 255, 256) && (tid & 63) == 0)
                changed[round % 3] = 1;
#ifdef SIMAPS_PHASE_STAMPS
            if (tid == 0 && round == 0) STAMP_NB(57);
            if (tid == 192 && round == 0) STAMP_NB(63);
#endif
            gs.sync();
#ifdef SIMAPS_PHASE_STAMPS
            if (tid == 0 && round == 0) STAMP_NB(78);
#endif
        }
        if (!changed[round % 3] || round >= max_rounds) {
            if ((tid & 255) == 0)  // cap hit: 1 << 20 (status bit 1)
                __hip_atomic_fetch_max(&sh.rounds, round >= max_rounds ? 1 << 20 : round + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef SIMAPS_PHASE_STAMPS
            if ((tid & 63) == 0 && blockIdx.x < MAX_STAMP_WG) g_stamps[blockIdx.x * NSTAMP + 64 + wave] = steps;
#endif
            break;
        }
    }
}

// group g: -inf (blocked) -> +inf; max reachable distance per source (sh.dmax, visible after the
// next workgroup barrier)
__device__ __forceinline__ void sssp_finish(Shared &sh, float *dist, int nsrc, const Group &g)
{
    const int cells = (sh.h + 2) * sssp_pitch(sh.w);
    for (int s = 0; s < nsrc; s++) {
        float m = -1.0f;
        for (int q = g.t; q < cells; q += g.n) {
            float &d = dist[s * DIST_FLOATS + q];
            if (d == -INFINITY) d = INFINITY;
            else if (d != INFINITY) m = fmaxf(m, d);
        }
        m = wave_max(m);
        if ((g.t & 63) == 0) sh.red[s][g.t >> 6] = m;
    }
    g.sync();
    if (g.t < nsrc) {
        float mm = sh.red[g.t][0];
        for (int k = 1; k < g.nw; k++) mm = fmaxf(mm, sh.red[g.t][k]);
        sh.dmax[g.t] = mm;
    }
}

// group g, after the rounds: the maximum reachable distance per source, read-only (envs.py:2288-2300:
// img = sp / 96, img[img < 0] = img.max(), img *= scale).  The distance phase scales the values it
// samples and reads blocked / unreachable / border cells (+-inf) as sh.unreach[s] =
// (max(sp) / 96) * scale (division and scaling are monotone: the max of the scaled values is the
// scaled max).
// one wave's part (threads t, t + n, ...) of the max finite value of D[0, cells); -1 if none
__device__ __forceinline__ float max_finite_part(const float *D, int cells, int t, int n)
{
    float m0 = -1.0f, m1 = -1.0f;
    int q = t;
    for (; q + n < cells; q += 2 * n) {  // two reads in flight per iteration
        const float v0 = D[q], v1 = D[q + n];
        m0 = fabsf(v0) != INFINITY ? fmaxf(m0, v0) : m0;
        m1 = fabsf(v1) != INFINITY ? fmaxf(m1, v1) : m1;
    }
    if (q < cells) {
        const float v0 = D[q];
        m0 = fabsf(v0) != INFINITY ? fmaxf(m0, v0) : m0;
    }
    return wave_max(fmaxf(m0, m1));
}

// after the group barrier that follows the partial maxima sh.red[s][0, parts)
__device__ __forceinline__ void sssp_max_final(Shared &sh, int nsrc, int parts, float scale, int t)
{
    if (t < nsrc) {
        float mm = sh.red[t][0];
        for (int k = 1; k < parts; k++) mm = fmaxf(mm, sh.red[t][k]);
        sh.dmax[t] = mm;
        sh.unreach[t] = (mm / 96.0f) * scale;
    }
}

__device__ __forceinline__ void sssp_max(Shared &sh, const float *dist, int nsrc, float scale, const Group &g)
{
    const int cells = (sh.h + 2) * sssp_pitch(sh.w);
    for (int s = 0; s < nsrc; s++) {
        const float m = max_finite_part(dist + s * DIST_FLOATS, cells, g.t, g.n);
        if ((g.t & 63) == 0) sh.red[s][g.t >> 6] = m;
    }
    g.sync();
    sssp_max_final(sh, nsrc, g.nw, scale, g.t);
}

// Split sweeps (one source, compile-time pitch; the single-kernel users, whose other waves idle): the
// two directions along the longer room side get KL waves each, the other two KS each, every wave one
// part of its direction's steps (sweep(..., part, nparts)).  Shorter sweeps per round, more rounds.
// Measured (tools/sssp_split_ab.sh, profiles/r3g_sssp_split_ab.jsonl): KL = KS = 2 takes 2-7 % off
// simaps_sssp_grid and simaps_sp_distance; KL = 2 alone, 3 alone, or 4 / 2 are slower than no split
// (their extra rounds outweigh the shorter ones).
#ifndef SIMAPS_SSSP_SPLIT_L
#define SIMAPS_SSSP_SPLIT_L 2
#endif
#ifndef SIMAPS_SSSP_SPLIT_S
#define SIMAPS_SSSP_SPLIT_S 2
#endif
constexpr int SPLIT_WAVES = 2 * (SIMAPS_SSSP_SPLIT_L + SIMAPS_SSSP_SPLIT_S);
static_assert(SPLIT_WAVES <= NT / 64, "split sweeps: one wave per part");
__device__ __forceinline__ void sssp_rounds_split(Shared &sh, float *dist)
{
    const int tid = threadIdx.x, wave = tid >> 6;
    const int h = sh.h, w = sh.w, pw = sssp_pitch(w);
    const int max_rounds = h * w + 16;
    const Group gs{tid, 64 * SPLIT_WAVES, sh.bar[2], SPLIT_WAVES};
    const int longd = w >= h ? 2 : 0;  // columns (right / left) sweep the w lines of a wide room
    const bool lw = wave < 2 * SIMAPS_SSSP_SPLIT_L;
    const int q = lw ? wave : wave - 2 * SIMAPS_SSSP_SPLIT_L;
    const int dir = (lw ? longd : 2 - longd) + (q & 1), part = q >> 1;
    const int nparts = lw ? SIMAPS_SSSP_SPLIT_L : SIMAPS_SSSP_SPLIT_S;
    if (lw) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(2);
    int *changed = sh.changed[0];
    int steps = 0;
    for (int round = 0;; round++) {
        if (tid == 0) changed[(round + 1) % 3] = 0;
        if (sh.src_ok[0] && sweep(dist, h, w, pw, dir, sh.dirty[0], steps, part, nparts) && (tid & 63) == 0 && !SSSP_CHECK)
            changed[round % 3] = 1;
        gs.sync();
        if (SSSP_CHECK) {
            if (sh.src_ok[0] && sssp_check(dist, h, w, pw, sh.dirty[0], tid, 64 * SPLIT_WAVES) && (tid & 63) == 0)
                changed[round % 3] = 1;
            gs.sync();
        }
        if (!changed[round % 3] || round >= max_rounds) {
            if (tid == 0)
                __hip_atomic_fetch_max(&sh.rounds, round >= max_rounds ? 1 << 20 : round + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
        }
    }
    __builtin_amdgcn_s_setprio(0);
}

// all threads (single-kernel users: sssp_grid_kernel, sp_distance_kernel)
__device__ __forceinline__ void sssp(Shared &sh, SsspScratch &S, float *dist, int nsrc)
{
    if (threadIdx.x < 16) (&sh.bar[0][0])[threadIdx.x] = 0u;
    sssp_init(sh, S, dist, nsrc, Group{(int)threadIdx.x, NT, nullptr, NT / 64});
    const int wave = threadIdx.x >> 6;
    if (SPLIT_WAVES > 4 && nsrc == 1 && sssp_pitch(sh.w) == 95) {
        if (wave < SPLIT_WAVES) sssp_rounds_split(sh, dist);
    } else if (wave < 4 * nsrc) sssp_rounds(sh, dist, nsrc, Group{(int)threadIdx.x, 256 * nsrc, sh.bar[0], 4 * nsrc});
    lds_barrier();
    sssp_finish(sh, dist, nsrc, Group{(int)threadIdx.x, NT, nullptr, NT / 64});
    lds_barrier();
}

// ------------------------------------------------------------------------------------------------
// Intention / history raster (Mapper._create_global_intention_or_history_map, envs.py:2302-2347)
// ------------------------------------------------------------------------------------------------
// enc: SIMAPS_ENC_* or 4 = history (ramp over the reversed history path)
// The per-robot segment table of one pass (robot k's lane; path_length accumulates sequentially).
// The first pass's table is built in the params phase, where its serial fp64 chain (sqrt, divide)
// overlaps the robot-rotation lanes instead of sitting on the render group's critical path.
__device__ __forceinline__ void seg_table(Shared &sh, const simaps_config &cfg, const simaps_robot *rb,
                                          const double *__restrict__ paths, int enc, int k, int me)
{
    int cnt = 0;
    const simaps_robot &r = rb[k];
    if (k != me && !r.idle && enc != SIMAPS_ENC_CIRCLE) {
        const double scale = cfg.intention_map_scale;
        const int off = enc == 4 ? r.history_off : r.intention_off;
        const int full = enc == 4 ? r.history_len : r.intention_len;
        const bool as_line = enc == SIMAPS_ENC_LINE && full >= 2;  // [path[0], path[-1]] (envs.py:2315-2316)
        const int len = as_line ? 2 : full;
        double L = 0.0;
        for (int i = 1; i < len && cnt < SEG_PER_ROBOT; i++) {
            const int ia = i - 1, ib = as_line ? full - 1 : i;
            const double sx = paths[2 * (off + ia)], sy = paths[2 * (off + ia) + 1];
            const double tx = paths[2 * (off + ib)], ty = paths[2 * (off + ib) + 1];
            const double dx = tx - sx, dy = ty - sy;
            const double seg_len = scale * sqrt(dx * dx + dy * dy);  // envs.py:2324, 2557-2558
            Seg &G = sh.seg[k * SEG_PER_ROBOT + cnt];
            pos_to_pix(sx, sy, cfg.H, cfg.W, G.si, G.sj);
            pos_to_pix(tx, ty, cfg.H, cfg.W, G.ti, G.tj);
            G.dr = abs(G.ti - G.si);
            G.dc = abs(G.tj - G.sj);
            G.n = (G.dr > G.dc ? G.dr : G.dc) + 1;
            G.last = (i == len - 1);
            // np.clip(np.linspace(1 - L, 1 - (L + seg), n), 0, 1) (envs.py:2335)
            G.start = 1 - L;
            G.stop = 1 - (L + seg_len);
            G.step = G.n > 1 ? (G.stop - G.start) / (G.n - 1) : 0.0;
            L += seg_len;
            cnt++;
        }
    }
    sh.seg_robot_cnt[k] = cnt;
}

// seg_table split over one lane per segment slot q = k * SEG_PER_ROBOT + (i - 1) (segment
// path[i - 1] -> path[i] of robot k): seg_geom (the pixels and the scaled length) in the params
// phase, seg_ramp (the running length L in path order, then the linspace ramp) after a barrier.
// Same fp64 operations in the same order as seg_table; a robot's segments no longer run serially.
__device__ __forceinline__ void seg_geom(Shared &sh, const simaps_config &cfg, const simaps_robot *rb,
                                         const double *__restrict__ paths, int enc, int q, int me)
{
    const int k = q / SEG_PER_ROBOT, i = q % SEG_PER_ROBOT + 1;
    const simaps_robot &r = rb[k];
    const bool on = k != me && !r.idle && enc != SIMAPS_ENC_CIRCLE;
    const int off = enc == 4 ? r.history_off : r.intention_off;
    const int full = enc == 4 ? r.history_len : r.intention_len;
    const bool as_line = enc == SIMAPS_ENC_LINE && full >= 2;  // [path[0], path[-1]] (envs.py:2315-2316)
    const int len = as_line ? 2 : full;
    if (i == 1) sh.seg_robot_cnt[k] = on && len >= 2 ? min(len - 1, SEG_PER_ROBOT) : 0;
    if (!on || i >= len) return;
    const int ia = i - 1, ib = as_line ? full - 1 : i;
    const double sx = paths[2 * (off + ia)], sy = paths[2 * (off + ia) + 1];
    const double tx = paths[2 * (off + ib)], ty = paths[2 * (off + ib) + 1];
    const double dx = tx - sx, dy = ty - sy;
    sh.seglen[q] = cfg.intention_map_scale * sqrt(dx * dx + dy * dy);  // envs.py:2324, 2557-2558
    Seg &G = sh.seg[q];
    pos_to_pix(sx, sy, cfg.H, cfg.W, G.si, G.sj);
    pos_to_pix(tx, ty, cfg.H, cfg.W, G.ti, G.tj);
    G.dr = abs(G.ti - G.si);
    G.dc = abs(G.tj - G.sj);
    G.n = (G.dr > G.dc ? G.dr : G.dc) + 1;
    G.last = (i == len - 1);
}
__device__ __forceinline__ void seg_ramp(Shared &sh, int q)
{
    const int k = q / SEG_PER_ROBOT, j = q % SEG_PER_ROBOT;
    if (j >= sh.seg_robot_cnt[k]) return;
    double L = 0.0;
    for (int m = 0; m < j; m++) L += sh.seglen[k * SEG_PER_ROBOT + m];
    Seg &G = sh.seg[q];
    // np.clip(np.linspace(1 - L, 1 - (L + seg), n), 0, 1) (envs.py:2335)
    G.start = 1 - L;
    G.stop = 1 - (L + sh.seglen[q]);
    G.step = G.n > 1 ? (G.stop - G.start) / (G.n - 1) : 0.0;
}

// max(v) into tile cell (a, b) and, for thick lines, its 4-neighbours: the grey dilation with disk(1)
// (envs.py:2343-2344) applied as a scatter at raster time, so a sample is one read.  The cross is
// symmetric, so scattering each line pixel into its cross equals dilating the raster; the tile's
// 1-px halo holds every neighbour of a crop pixel.
__device__ __forceinline__ void tile_put(unsigned *tu, int a, int b, float v, int thick)
{
    const unsigned u = __float_as_uint(v);  // v > 0: the uint order is the float order
    if ((unsigned)a < (unsigned)TILE && (unsigned)b < (unsigned)TILE) atomicMax(&tu[a * TILE + b], u);
    if (thick > 1) {
        if ((unsigned)(a - 1) < (unsigned)TILE && (unsigned)b < (unsigned)TILE) atomicMax(&tu[(a - 1) * TILE + b], u);
        if ((unsigned)(a + 1) < (unsigned)TILE && (unsigned)b < (unsigned)TILE) atomicMax(&tu[(a + 1) * TILE + b], u);
        if ((unsigned)a < (unsigned)TILE && (unsigned)(b - 1) < (unsigned)TILE) atomicMax(&tu[a * TILE + b - 1], u);
        if ((unsigned)a < (unsigned)TILE && (unsigned)(b + 1) < (unsigned)TILE) atomicMax(&tu[a * TILE + b + 1], u);
    }
}

// Rasterise one pass into the tile (max of line values per pixel).  Zeroes the tile and, unless
// the params phase already did, builds the segment table; two group barriers.
// (zeroed: the sweep track already zeroed the tile and the table exists: no zeroing, no barrier)
__device__ __forceinline__ void raster_lines(Shared &sh, float *tile, const simaps_config &cfg, const simaps_robot *rb,
                             const double *__restrict__ paths, int enc, bool have_table, const Group &g,
                             bool zeroed = false)
{
    const int tid = g.t, lane = threadIdx.x & 63, wave = g.t >> 6, nwaves = g.n >> 6;
    unsigned *tu = reinterpret_cast<unsigned *>(tile);
    const float scale_f = (float)cfg.intention_map_scale;
    const int thick = cfg.intention_map_line_thickness;
    if (!(zeroed && have_table)) {
        uint4 *tz = reinterpret_cast<uint4 *>(tile);
        for (int k = tid; k < TILE * TILE / 4; k += g.n) tz[k] = uint4{0u, 0u, 0u, 0u};
        if (!have_table && tid < sh.nr) seg_table(sh, cfg, rb, paths, enc, tid, sh.me);
        g.sync();
    }
    static_assert(TILE * TILE % 4 == 0, "tile zeroing");
    if (tid == 0 && have_table) STAMP_NB(60);
    const int ti0 = sh.pi - TILE_HALF, tj0 = sh.pj - TILE_HALF;
    if (enc == SIMAPS_ENC_CIRCLE) {
        if (tid < sh.nr && tid != sh.me && !sh.rob[tid].idle) {
            const int a = sh.rob[tid].tpi - ti0, b = sh.rob[tid].tpj - tj0;
            tile_put(tu, a, b, scale_f, thick);
        }
    } else {
        // The segments' pixels, cut to the tile rows / columns along the major axis (a pixel outside
        // them only reaches the unsampled halo), in chunks of 64 (one per lane), dealt round-robin
        // to the waves.  Every wave builds the chunk ranges itself: lane q (and q + 64) holds slot
        // q's first in-tile pixel and chunk count; an inclusive scan gives each slot's chunk range.
        static_assert(SIMAPS_MAX_ROBOTS * SEG_PER_ROBOT <= 128, "two slots per lane");
        static_assert(320 + SIMAPS_MAX_ROBOTS * SEG_PER_ROBOT <= 512, "one params-phase lane per segment slot");
        const int total = sh.nr * SEG_PER_ROBOT;
        int t_lo[2], nch[2], c_end[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int q = lane + 64 * h;
            t_lo[h] = 0;
            nch[h] = 0;
            if (q < total && q % SEG_PER_ROBOT < sh.seg_robot_cnt[q / SEG_PER_ROBOT]) {
                const Seg &G = sh.seg[q];
                const int npix = G.last ? G.n : G.n - 1;  // non-final segments drop their last pixel
                const bool steep = G.dr > G.dc;
                const int m0 = steep ? G.si : G.sj, m1 = steep ? G.ti : G.tj, lo = steep ? ti0 : tj0;
                int a0, a1;  // t range whose major coordinate m0 +- t lies in [lo, lo + TILE)
                if (m1 >= m0) { a0 = lo - m0; a1 = lo + TILE - 1 - m0; }
                else { a0 = m0 - (lo + TILE - 1); a1 = m0 - lo; }
                a0 = max(a0, 0);
                a1 = min(a1, npix - 1);
                t_lo[h] = a0;
                nch[h] = a1 >= a0 ? ((a1 - a0) >> 6) + 1 : 0;
            }
            int x = nch[h];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            c_end[h] = x;
        }
        const int tot0 = __builtin_amdgcn_readlane(c_end[0], 63);
        c_end[1] += tot0;
        const int nchunks = __builtin_amdgcn_readlane(c_end[1], 63);
        for (int c = wave; c < nchunks; c += nwaves) {
            const int h = c < tot0 ? 0 : 1;
            const uint64_t m = __ballot(h == 0 ? (c < c_end[0]) : (c < c_end[1]));  // c_end is monotone
            const int L = __builtin_amdgcn_readfirstlane(__builtin_ctzll(m));
            const int q = L + 64 * h;
            const int cbeg = __builtin_amdgcn_readlane(h == 0 ? c_end[0] - nch[0] : c_end[1] - nch[1], L);
            const int t0 = __builtin_amdgcn_readlane(h == 0 ? t_lo[0] : t_lo[1], L);
            const Seg &G = sh.seg[q];
            const int npix = G.last ? G.n : G.n - 1;
            const bool steep = G.dr > G.dc;
            const int major = steep ? G.dr : G.dc, minor = steep ? G.dc : G.dr;
            const int smaj = steep ? (G.ti - G.si > 0 ? 1 : -1) : (G.tj - G.sj > 0 ? 1 : -1);
            const int smin = steep ? (G.tj - G.sj > 0 ? 1 : -1) : (G.ti - G.si > 0 ? 1 : -1);
            const int t = t0 + (c - cbeg) * 64 + lane;
            if (t < npix) {
                int pr, pc;
                if (t == G.n - 1) {  // skimage: rr[dc] = r1, cc[dc] = c1
                    pr = G.ti;
                    pc = G.tj;
                } else {  // closed-form Bresenham: minor steps k_t = floor((2*minor*t + major) / (2*major))
                    const int kt = (2 * minor * t + major) / (2 * major);
                    if (steep) { pr = G.si + smaj * t; pc = G.sj + smin * kt; }
                    else { pc = G.sj + smaj * t; pr = G.si + smin * kt; }
                }
                float v;
                if (enc == SIMAPS_ENC_BINARY || enc == SIMAPS_ENC_LINE) {
                    v = scale_f;
                } else {
                    double y = (t == G.n - 1 && G.n > 1) ? G.stop : (G.n > 1 ? (double)t * G.step + G.start : G.start);
                    y = y < 0.0 ? 0.0 : (y > 1.0 ? 1.0 : y);
                    v = (float)y;
                }
                const int a = pr - ti0, b = pc - tj0;
                if (v > 0.0f) tile_put(tu, a, b, v, thick);
            }
        }
    }
    if (tid == 0 && have_table) STAMP_NB(61);
    g.sync();
}

// The raster tile aliases the cspace scratch: the render group waits until the sweep group has
// released it (sweep_track; set from the start when no group builds a cspace).  Lane 0 of each wave
// polls; the acquire fence orders the wave's later tile accesses after the release.
__device__ __forceinline__ void wait_scratch(Shared &sh)
{
    if ((threadIdx.x & 63) == 0) {
        unsigned spins = 0;
        while (!__hip_atomic_load(&sh.scratch_free, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) {  // never in a correct run: flag (SIMAPS_FAULT_TIMEOUT) and fall through
                __hip_atomic_store(&sh.bar[1][2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                break;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ float tile_sample(const float *tile, int gi, int gj, int pi, int pj)
{
    return tile[(gi - pi + TILE_HALF) * TILE + (gj - pj + TILE_HALF)];  // dilated at raster time (tile_put)
}

// ------------------------------------------------------------------------------------------------
// The fused per-agent kernel
// ------------------------------------------------------------------------------------------------

struct RenderCtx {
    const simaps_config &cfg;
    Shared &sh;
    float *out;
    int C, n;
    __device__ __forceinline__ void put(int ch, int p, float v) const
    {
        unsigned idx = cfg.layout_chw ? ch * LW * LW + p : p * C + ch;  // < 96 * 96 * C: 32-bit
        asm volatile("" : "+v"(idx));  // computed at the store: no per-pixel offsets hoisted across passes
        // 32-bit byte offset from an SGPR base: one VGPR per address (saddr form), no 64-bit adds
        *reinterpret_cast<float *>(reinterpret_cast<char *>(out) + idx * 4u) = v;
    }
    // chw only: 4 consecutive pixels p .. p + 3 (p % 4 == 0) of channel ch, one 16-byte store
    __device__ __forceinline__ void put4(int ch, int p, float4 v) const
    {
        unsigned idx = ch * LW * LW + p;
        asm volatile("" : "+v"(idx));
        *reinterpret_cast<float4 *>(reinterpret_cast<char *>(out) + idx * 4u) = v;
    }
};

// A robot's stamp geometry (Mapper._create_global_robot_map, envs.py:2251-2276): the scipy rotate of
// its class mask (angle = degrees(heading) - 90), the placement pixel - S // 2, a conservative box of
// global pixels outside which the rotated mask is surely 0, its robot-code bits and seg value.  (Also
// the global-maps debug kernel's, global_maps.h.)
__device__ __forceinline__ void robot_params(RobotP &P, const simaps_robot &r, const simaps_config &cfg, const Geometry &geo,
                                             int H, int W)
{
    const Rot R = rot_params(LW, r.heading * RAD_TO_DEG - 90.0, cfg.rotate_rounding == SIMAPS_ROT_PLAIN);
    P.c = R.c; P.s = R.s; P.f0 = R.f0; P.f1 = R.f1; P.S0 = R.S0; P.S1 = R.S1;
    int pi, pj;
    pos_to_pix(r.x, r.y, H, W, pi, pj);
    P.st_i = pi - R.S0 / 2;
    P.st_j = pj - R.S1 / 2;
    P.type = r.type; P.lifting = r.lifting; P.idle = r.idle; P.group = r.group_index;
    P.x = r.x; P.y = r.y; P.tx = r.target_x; P.ty = r.target_y;
    pos_to_pix(r.target_x, r.target_y, H, W, P.tpi, P.tpj);
    {   // conservative prefilter box: inverse-rotate the mask's nonzero window (+-2 px)
        const int st = geo.mask_start[r.type], wd = geo.mask_width[r.type];
        const double lo0 = st - (r.type == SIMAPS_LIFTING ? geo.cube_w : 0) - 1.0, hi0 = st + wd + 1.0;
        const double lo1 = st - 1.0, hi1 = st + wd + 1.0;
        double mn0 = 1e30, mx0 = -1e30, mn1 = 1e30, mx1 = -1e30;
        for (int q = 0; q < 4; q++) {
            const double a = ((q & 1) ? hi0 : lo0) - R.f0, b = ((q & 2) ? hi1 : lo1) - R.f1;
            const double o0 = R.c * a - R.s * b, o1 = R.s * a + R.c * b;
            mn0 = fmin(mn0, o0); mx0 = fmax(mx0, o0); mn1 = fmin(mn1, o1); mx1 = fmax(mx1, o1);
        }
        P.bi0 = max(P.st_i, P.st_i + (int)floor(mn0) - 2);
        P.bi1 = min(P.st_i + R.S0 - 1, P.st_i + (int)ceil(mx0) + 2);
        P.bj0 = max(P.st_j, P.st_j + (int)floor(mn1) - 2);
        P.bj1 = min(P.st_j + R.S1 - 1, P.st_j + (int)ceil(mx1) + 2);
        P.bi1 = min(P.bi1, P.bi0 + 31);  // the window is <= 17 x 13 px: its rotated box fits 32 x 32
        P.bj1 = min(P.bj1, P.bj0 + 31);
    }
    P.seg_val = (float)((r.group_index + 1 + 4) / 8.0);  // SEG_VALUES['robot_group_{g+1}'] (envs.py:1885-1889)
    P.code0 = (1u << r.group_index) | (r.type != SIMAPS_LIFTING ? 1u << 5 : (!r.lifting ? 1u << 4 : 0u));}

// Mapper._get_intention_channels (envs.py:2349-2378), the per-agent part: robots ordered by
// distance (np.argsort -> stable insertion sort) and the nonspatial (dist * sin, dist * cos) pairs.
// One thread, in the params phase (fp64 libm calls need registers the render phase does not have).
__device__ __forceinline__ void intention_channel_order(Shared &sh, const simaps_config &cfg, const simaps_robot *rb)
{
    const int nr = sh.nr;
    double dd[SIMAPS_MAX_ROBOTS];
    const RobotP &M = sh.rob[sh.me];
    for (int q = 0; q < nr; q++) {
        const double dx = sh.rob[q].x - M.x, dy = sh.rob[q].y - M.y;
        dd[q] = sqrt(dx * dx + dy * dy);
        int j = q;
        while (j > 0 && dd[sh.order[j - 1]] > dd[q]) { sh.order[j] = sh.order[j - 1]; j--; }
        sh.order[j] = q;
    }
    if (!cfg.intention_channel_spatial) {
        int c2 = 0;
        for (int q = 0; q < nr; q++) {
            const int k = sh.order[q];
            if (k == sh.me) continue;
            const RobotP &R = sh.rob[k];
            double rel0 = 0.0, rel1 = 0.0;
            if (!R.idle) {
                const double dx = R.tx - M.x, dy = R.ty - M.y;
                const double dist_t = sqrt(dx * dx + dy * dy);
                const double th = rb[sh.me].heading - atan2(R.ty - M.y, R.tx - M.x);
                rel0 = dist_t * sin(th);
                rel1 = dist_t * cos(th);
            }
            sh.nonsp[c2++] = (float)(cfg.intention_channel_nonspatial_scale * rel0);
            sh.nonsp[c2++] = (float)(cfg.intention_channel_nonspatial_scale * rel1);
        }
    }
}

// Channels that do not need the shortest-path maps, rendered by group g:
// overhead (0), robot (1), history / intention maps, baseline intention channels.
//
// Sample indices (Mapper._get_local_map, envs.py:2200-2211; rot_src): each output pixel's source
// index in the crop is computed once per pixel and reused by every channel and the distance phase.
// NPT: output pixels per render thread (18 / 12 / 9 for 8 / 12 / 16 render waves), a compile-time
// constant so every pixel loop is exact (no bounds tests) and its index math folds.
template <int NPT>
__device__ __forceinline__ void render_maps(const RenderCtx &rc, const Group &g, const Geometry &geo, const float *__restrict__ ovh,
                            const simaps_robot *rb, const double *__restrict__ paths, float *tile,
                            const uint8_t *cmap, bool early_tile, bool tail_cells, float *smem_dist)
{
    const simaps_config &cfg = rc.cfg;
    Shared &sh = rc.sh;
    const int nr = sh.nr, W = cfg.W, H = cfg.H;
    constexpr int NP = LW * LW;
    const int ci0 = __builtin_amdgcn_readfirstlane(sh.pi - HALF_CROP);
    const int cj0 = __builtin_amdgcn_readfirstlane(sh.pj - HALF_CROP);
    // the sample index of each of this thread's output pixels (fast fp32 path, exact fp64 fallback),
    // packed 2 per register: crop-relative (row << 8 | col), 0xffff = outside (cval)
    constexpr int MAXPG = NPT;
    constexpr int GN = NP / NPT;  // == g.n
    static_assert(GN * NPT == NP && GN % 64 == 0, "render group split");
    // item k of a thread: pixel g.t + k * GN (a wave item = 64 consecutive pixels: whole-line stores).
    // (2 x 32 pixel blocks -- half the cache lines per rotated overhead gather, still whole-line
    // stores -- measured 6-10 % slower in every config: round 2 A/B)
    auto rpix = [&](int k) { return g.t + k * GN; };
    uint32_t gqp[(MAXPG + 1) / 2];
    {   // every pixel exactly in fp64 (rot_src's arithmetic, branch-free): cheaper than an fp32 fast path
        // whose rounding-band fallback diverges in most waves
        const Rot R = sh.rot;
        const int oa = R.S0 / 2 - LW / 2, ob = R.S1 / 2 - LW / 2;
        const double hd = CROP - 1;
#pragma unroll
        for (int k = 0; k < MAXPG; k++) {
            const int p = rpix(k), a = p / LW, b = p - (p / LW) * LW;
            const double d0 = a + oa, d1 = b + ob;
            const double s0 = (d0 * R.c + d1 * R.s) + R.f0, s1 = (d0 * (-R.s) + d1 * R.c) + R.f1;
            const int in = (s0 >= 0.0) & (s0 <= hd) & (s1 >= 0.0) & (s1 <= hd);
            const int i0 = (int)floor(s0 + 0.5), i1 = (int)floor(s1 + 0.5);
            const int inmap = ((unsigned)(ci0 + i0) < (unsigned)H) & ((unsigned)(cj0 + i1) < (unsigned)W);
            const uint32_t v = (in & inmap) ? (((uint32_t)i0 << 8) | (uint32_t)i1) : 0xffffu;
            if (k & 1) gqp[k >> 1] |= v << 16;
            else gqp[k >> 1] = v | (k == MAXPG - 1 ? 0xffff0000u : 0u);
        }
#ifdef SIMAPS_PHASE_STAMPS
        if (g.t == 0) {
            asm volatile("" ::"v"(gqp[0]), "v"(gqp[8]));
            STAMP_NB(40);
        }
#endif
    }
    auto gq_v = [&](int k) -> uint32_t { return (gqp[k >> 1] >> ((k & 1) * 16)) & 0xffffu; };
    // channel index after overhead / robot / distance channels (envs.py:2071-2113 order)
    int ch = 1 + !!cfg.use_robot_map + !!cfg.use_distance_to_receptacle_map + !!cfg.use_shortest_path_to_receptacle_map +
             !!cfg.use_shortest_path_map;
    // history / intention passes, rasterised into the LDS tile (the first pass's segment table was
    // built in the params phase)
    int encs[2], npass = 0;
    if (cfg.use_history_map) encs[npass++] = 4;
    if (cfg.use_intention_map) encs[npass++] = cfg.intention_map_encoding;
    const int thick = cfg.intention_map_line_thickness;
#ifdef SIMAPS_PHASE_STAMPS
    if (g.t == 0) {
        asm volatile("" ::"v"(gqp[0]), "v"(gqp[8]));
        STAMP_NB(41);
    }
#endif
    // every overhead gather of the thread in flight at once; the robot-code lookups run meanwhile
    float ovv[MAXPG];
#pragma unroll
    for (int k = 0; k < MAXPG; k++) {
        uint32_t v = gq_v(k);
        asm volatile("" : "+v"(v));  // nothing computed here is shared with (kept alive for) later passes
        // branch-free, 32-bit offsets (SGPR base): pixels outside the crop load cell 0, ignored later
        const int idx = (ci0 + (int)(v >> 8)) * W + (cj0 + (int)(v & 0xffu));
        ovv[k] = *reinterpret_cast<const float *>(reinterpret_cast<const char *>(ovh) + (unsigned)(v != 0xffffu ? idx : 0) * 4u);
    }
    if (g.t == 0) STAMP_NB(42);
    // overhead / robot channels (Mapper._create_global_overhead_map / _create_global_robot_map,
    // envs.py:2244-2276) from the crop's robot-code map (stamps phase): one LDS byte per pixel.
    // Bit g of the code = seg value (g + 5) / 8 (SEG_VALUES robot_group_{g+1}), bit 4 = 0.5,
    // bit 5 = 1.0 (lifted-cube mask); the max over robots is the highest bit.  Outside pixels
    // (0xffff) read the zero guard after the map.
    unsigned codes[(MAXPG + 3) / 4] = {};
#pragma unroll
    for (int k = 0; k < MAXPG; k++) {
        const uint32_t v = gq_v(k);
        const unsigned m = cmap[v != 0xffffu ? (int)(v >> 8) * CROP + (int)(v & 0xffu) : CROP * CROP];
        codes[k >> 2] |= m << (8 * (k & 3));
    }
    if (g.t == 0) STAMP_NB(14);
#pragma unroll
    for (int k = 0; k < MAXPG; k++) {
        const int p = rpix(k);
        uint32_t v = gq_v(k);
        asm volatile("" : "+v"(v));
        const unsigned m = (codes[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const unsigned ms = m & 0xfu, mr = m >> 4;
        const float vseg = ms ? (float)(31 - __builtin_clz(ms) + 5) * 0.125f : 0.0f;
        const float vrob = (mr & 2u) ? 1.0f : ((mr & 1u) ? 0.5f : 0.0f);
        const float vov = vseg > 0.0f ? vseg : (v != 0xffffu ? ovv[k] : 0.0f);
        rc.put(0, p, vov);
        if (cfg.use_robot_map) rc.put(1, p, vrob);
    }
    if (g.t == 0) STAMP_NB(11);
    // sample one rasterised pass into channel c (then the tile may be reused)
    auto sample_pass = [&](int c, bool last) {
        if (g.t == 0) STAMP_NB(12);
#pragma unroll
        for (int k = 0; k < MAXPG; k++) {
            const int p = rpix(k);
            uint32_t v = gq_v(k);
            asm volatile("" : "+v"(v));
            rc.put(c, p, v != 0xffffu ? tile_sample(tile, ci0 + (int)(v >> 8), cj0 + (int)(v & 0xffu), sh.pi, sh.pj) : 0.0f);
        }
        if (!(last && tail_cells)) g.sync();  // the tile is overwritten next (raster pass or tables)
    };
    // history / intention passes, rasterised into the LDS tile, which overwrites the code map (every
    // render wave has read it: group barrier) and the sweep track's scratch (wait for its release)
    if (npass > 0) {
        // early_tile: the code map lies outside the tile and the sweep track zeroed the tile when it
        // released its scratch -- no barrier; else every render wave must be done with the code map
        if (!early_tile) g.sync();
        wait_scratch(sh);
        if (g.t == 0) STAMP_NB(62);
        raster_lines(sh, tile, cfg, rb, paths, encs[0], true, g, early_tile);
        if (g.t == 0) STAMP_NB(13);
        sample_pass(ch, npass == 1);
    }
    // the second history / intention pass (history + intention configs)
    if (npass > 1) {
        raster_lines(sh, tile, cfg, rb, paths, encs[1], false, g);
        sample_pass(ch + 1, true);
    }
    ch += npass;
    // baseline intention channels (Mapper._get_intention_channels, envs.py:2349-2378)
    if (cfg.use_intention_channels) {  // sh.order / sh.nonsp: intention_channel_order (params phase)
        int c2 = 0;
        const float scale_f = (float)cfg.intention_map_scale;
        for (int q = 0; q < nr; q++) {
            const int kq = sh.order[q];
            if (kq == sh.me) continue;
            if (cfg.intention_channel_spatial) {
                const RobotP &R = sh.rob[kq];
#pragma unroll
                for (int k = 0; k < MAXPG; k++) {
                    const int p = rpix(k);
                    const uint32_t v = gq_v(k);
                    float val = 0.0f;
                    if (v != 0xffffu && !R.idle) {
                        const int di = abs(ci0 + (int)(v >> 8) - R.tpi), dj = abs(cj0 + (int)(v & 0xffu) - R.tpj);
                        const bool hit = thick > 1 ? (di + dj <= 1) : (di == 0 && dj == 0);
                        val = hit ? scale_f : 0.0f;
                    }
                    rc.put(ch, p, val);
                }
                ch++;
            } else {
                for (int e = 0; e < 2; e++, ch++, c2++)
                    for (int k = 0; k < MAXPG; k++) rc.put(ch, rpix(k), sh.nonsp[c2]);
            }
        }
    }
    // hand the sample indices to the distance phase: crop-relative (row << 8 | col), 0xffff = cval
    // (the tile region is free: every raster pass ended with a group barrier; without one, wait for
    // every render wave's code-map reads and for the sweep track's scratch release)
    // and the byte offset of each pixel's distance-array cell (0 = outside the room rect: the border
    // cell, +-inf; CVAL_OFF = cval), so the 16-wave distance phase does no index math.  tail_cells
    // (small rooms, no Euclidean map): only the cell table, in the unused tail of distance array 0,
    // which no one else touches -- no barrier, no wait
    if (tail_cells) {
        uint16_t *tc = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(smem_dist) + tail_cells_off(cfg.room_h, cfg.room_w));
        const int ri0 = ci0 - cfg.room_i0, rj0 = cj0 - cfg.room_j0, pw = sssp_pitch(cfg.room_w);
        const unsigned rh = cfg.room_h, rw = cfg.room_w;
#pragma unroll
        for (int k = 0; k < MAXPG; k++) {
            const uint32_t v = gq_v(k);
            const int r = ri0 + (int)(v >> 8), c = rj0 + (int)(v & 0xffu);
            const int in = (int)((unsigned)r < rh) & (int)((unsigned)c < rw);
            tc[rpix(k)] = (uint16_t)(v == 0xffffu ? CVAL_OFF : (uint32_t)(((r + 1) * pw + c + 1) & -in) * 4u);
        }
        return;
    }
    if (npass == 0) {
        if (!early_tile) g.sync();
        wait_scratch(sh);
    }
    uint16_t *tab = reinterpret_cast<uint16_t *>(tile);
    const int ri0 = ci0 - cfg.room_i0, rj0 = cj0 - cfg.room_j0, pw = sssp_pitch(cfg.room_w);
    const unsigned rh = cfg.room_h, rw = cfg.room_w;
#pragma unroll
    for (int k = 0; k < MAXPG; k++) {
        const uint32_t v = gq_v(k);
        const int r = ri0 + (int)(v >> 8), c = rj0 + (int)(v & 0xffu);
        const int in = (int)((unsigned)r < rh) & (int)((unsigned)c < rw);
        const uint32_t cell = v == 0xffffu ? CVAL_OFF : (uint32_t)(((r + 1) * pw + c + 1) & -in) * 4u;
        tab[rpix(k)] = (uint16_t)v;
        tab[NP + rpix(k)] = (uint16_t)cell;
    }
}

constexpr int PPT = (LW * LW) / NT;  // 9 output pixels per thread
static_assert(PPT * NT == LW * LW, "pixel split");

// Distance channels (all 16 waves): Euclidean map, then shortest-path maps; local -= local.min()
// (envs.py:2213-2216), so every value is kept in registers until the block minimum is known.
// A finite dist[] value d becomes (d / 96) * scale here; blocked, unreachable and border cells hold
// +-inf and read as the "unreachable" value (sssp_max), which is also the value of every global pixel
// outside the room rect, so an out-of-rect pixel just reads cell 0 (a border corner).  Everything the
// per-pixel loop needs from `sh` is read once into registers: the loop is straight-line code.
__device__ __forceinline__ void render_distance_channels(const RenderCtx &rc, const simaps_env &ev, const float *dist, int nsrc,
                                         const uint16_t *tab, const uint16_t *tcell)
{
    const simaps_config &cfg = rc.cfg;
    Shared &sh = rc.sh;
    const int tid = threadIdx.x, H = cfg.H, W = cfg.W;
    const int has_eu = cfg.use_distance_to_receptacle_map ? 1 : 0;
    const int nd = has_eu + nsrc;
    if (nd == 0) return;
    const int ch = 1 + !!cfg.use_robot_map;
    // Pixels of this thread: two aligned quads 4 * (tid + j * NT) + [0, 4) (in the chw layout one
    // 16-byte store per channel each) and the single pixel 8 * NT + tid.
    static_assert(PPT == 9, "two quads + one pixel per thread");
    auto pix = [&](int k) { return k < 8 ? 4 * (tid + (k >> 2) * NT) + (k & 3) : 8 * NT + tid; };
    // per pixel: the byte offset of its distance-array cell (0 = outside the rect: the border cell,
    // +-inf), CVAL_OFF outside the rotated crop (render_maps' second table), used as the LDS address
    unsigned coff[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        coff[k] = __builtin_nontemporal_load(tcell + pix(k));  // one ds_read_u16 each, no unpacking
    }
    // vals[0]: Euclidean map (first, envs.py:2083-2084) if present; vals[1 + s]: source s.  Each
    // branch is wave-uniform and outside the pixel loop, so a channel's loads issue back to back.
    float vals[3][PPT];
    float mins[3] = {INFINITY, INFINITY, INFINITY};
    if (has_eu) {  // envs.py:2278-2286
        const float eus = (float)cfg.distance_to_receptacle_map_scale;
        const int ci0 = __builtin_amdgcn_readfirstlane(sh.pi - HALF_CROP);
        const int cj0 = __builtin_amdgcn_readfirstlane(sh.pj - HALF_CROP);
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned sv = tab[pix(k)];
            const int gi = ci0 + (int)(sv >> 8), gj = cj0 + (int)(sv & 0xffu);
            const double px = ((gj + 0.5) - (double)W / 2) / PPM, py = ((double)H / 2 - (gi + 0.5)) / PPM;
            const double dx = ev.receptacle_x - px, dy = ev.receptacle_y - py;
            const float v = coff[k] == CVAL_OFF ? 0.0f : (float)sqrt(dx * dx + dy * dy) * eus;
            vals[0][k] = v;
            mins[0] = fminf(mins[0], v);
        }
    }
    // Source channels (envs.py:2288-2300): a finite distance d -> div96(d) * scale, two pixels per
    // packed-fp32 op; +-inf -> NaN there (inf - inf in div96), which fminf against the unreachable
    // value replaces (with |scale|, un = div96(max finite) * |scale| bounds every finite value; a
    // negative scale flips the signs afterwards, exactly); cval -> +0.
    const float scale = (float)cfg.shortest_path_map_scale;
    const bool neg = scale < 0.0f;
    const float as = fabsf(scale);
#pragma unroll
    for (int s = 0; s < 2; s++) {
        if (s >= nsrc) continue;
        typedef __attribute__((address_space(3))) const char lds_cchar;
        lds_cchar *D = (lds_cchar *)(dist + s * DIST_FLOATS);
        const float un = neg ? -sh.unreach[s] : sh.unreach[s];
        float v[PPT + 1];
#pragma unroll
        for (int k = 0; k < PPT; k++) v[k] = *(const lds_float *)(D + coff[k]);
        v[PPT] = 0.0f;
#pragma unroll
        for (int k = 0; k < PPT; k += 2) {
            const f32x2 d = {v[k], v[k + 1]};
            const f32x2 q0 = d * (1.0f / 96.0f);
            const f32x2 e = __builtin_elementwise_fma(-q0, f32x2{96.0f, 96.0f}, d);
            const f32x2 x = __builtin_elementwise_fma(e, f32x2{1.0f / 96.0f, 1.0f / 96.0f}, q0) * as;
            vals[1 + s][k] = coff[k] == CVAL_OFF ? 0.0f : fminf(x.x, un);
            if (k + 1 < PPT) vals[1 + s][k + 1] = coff[k + 1] == CVAL_OFF ? 0.0f : fminf(x.y, un);
        }
        if (neg) {
#pragma unroll
            for (int k = 0; k < PPT; k++) vals[1 + s][k] = coff[k] == CVAL_OFF ? 0.0f : -vals[1 + s][k];
        }
#pragma unroll
        for (int k = 0; k < PPT; k++) mins[1 + s] = fminf(mins[1 + s], vals[1 + s][k]);
    }
    if (tid == 0) STAMP_NB(16);
#pragma unroll
    for (int q = 0; q < 3; q++) {
        if (q == 0 ? !has_eu : q > nsrc) continue;
        const float m = wave_min(mins[q]);
        if ((tid & 63) == 0) sh.red[q][tid >> 6] = m;
    }
    lds_barrier();
    if (tid == 0) STAMP_NB(17);
#pragma unroll
    for (int q = 0; q < 3; q++) {
        if (q == 0 ? !has_eu : q > nsrc) continue;
        float mm = sh.red[q][0];
        for (int k = 1; k < NT / 64; k++) mm = fminf(mm, sh.red[q][k]);
        mins[q] = mm;
    }
#pragma unroll
    for (int q = 0; q < 3; q++) {
        if (q == 0 ? !has_eu : q > nsrc) continue;
        const int c = ch + q - 1 + has_eu;
        const float m = mins[q];
        if (cfg.layout_chw) {
#pragma unroll
            for (int j = 0; j < 2; j++)
                rc.put4(c, 4 * (tid + j * NT), make_float4(vals[q][4 * j] - m, vals[q][4 * j + 1] - m,
                                                            vals[q][4 * j + 2] - m, vals[q][4 * j + 3] - m));
            rc.put(c, 8 * NT + tid, vals[q][8] - m);
        } else {
#pragma unroll
            for (int k = 0; k < PPT; k++) rc.put(c, pix(k), vals[q][k] - m);
        }
    }
}

// group g, after sssp_finish and before sssp_scale (debug only): the raw distances of both sources,
// unreachable / blocked -> -1 (GridGraph.shortest_path_image)
__device__ __forceinline__ void dump_dist(const Shared &sh, const float *dist, float *out, const Group &g)
{
    const int hw = sh.h * sh.w;
    for (int k = g.t; k < 2 * hw; k += g.n) {
        const int which = k / hw, rem = k % hw;
        const int s = sh.sp_slot[which];
        float v = -1.0f;
        if (s >= 0) {
            v = dist[s * DIST_FLOATS + (rem / sh.w + 1) * sssp_pitch(sh.w) + rem % sh.w + 1];
            if (v == __int_as_float(INF_BITS)) v = -1.0f;
        }
        out[k] = v;
    }
}

// The cspace / SSSP track of get_state_kernel (group g = waves [0, 64 * G)): occupancy window ->
// cspace (OccupancyMap.update, envs.py:2453-2454) -> snapped sources (envs.py:2514-2517, 2523-2524)
// -> distance arrays; then the cspace scratch is released to the render group's raster tile and
// the sweeps run to the fixpoint (GridGraph._spfa, pyx:69-114), finish and scale in place.
template <int G>
__device__ __forceinline__ void sweep_track(Shared &sh, SsspScratch &S, float *dist, const simaps_config &cfg,
                                            const Geometry &geo, const simaps_agent &ag, const simaps_env &ev,
                                            const simaps_robot *__restrict__ robots,
                                            const uint8_t *__restrict__ occupancy, int nsrc, const simaps_debug &dbg,
                                            int n, const Group &g, bool zero_tile)
{
    const int t = g.t, H = cfg.H, W = cfg.W;
    const int h = cfg.room_h, w = cfg.room_w;
    OccLoad4<G> occ4;  // issued first: they depend on the map slot only
    const bool use4 = occ4_ok(H, W, cfg.room_j0);  // dword loads: 9 (G = 512) / 18 (G = 256) per thread
#ifdef SIMAPS_PHASE_STAMPS
    if (t == 0 && ag.map_slot >= 0) STAMP_NB(43);  // the agent record has landed
#endif
    const uint8_t *occ = occupancy + (size_t)ag.map_slot * H * W;
    if (use4) cspace_load4<G>(occ4, occ, H, W, cfg.room_i0, cfg.room_j0, h, t);
    const simaps_robot *rb = robots + ev.robot_off;
    if (t == 0) {
        sh.h = h;
        sh.w = w;
        sh.i0 = cfg.room_i0;
        sh.j0 = cfg.room_j0;
        int ns = 0;
        sh.sp_slot[0] = sh.sp_slot[1] = -1;
        if (cfg.use_shortest_path_to_receptacle_map) {
            pos_to_pix(ev.receptacle_x, ev.receptacle_y, H, W, sh.src_q[ns][0], sh.src_q[ns][1]);
            sh.sp_slot[0] = ns++;
        }
        if (cfg.use_shortest_path_map) {
            pos_to_pix(rb[ag.robot].x, rb[ag.robot].y, H, W, sh.src_q[ns][0], sh.src_q[ns][1]);
            sh.sp_slot[1] = ns++;
        }
        sh.nsrc = ns;
    }
    build_cspace<G>(S, nullptr, h, w, geo.cspace_r[rb[ag.robot].type], g, dist, nsrc, use4 ? &occ4 : nullptr, occ, H, W,
                    cfg.room_i0, cfg.room_j0);  // (its first sync publishes sh)
    if (t == 0) STAMP_NB(2);
    if (dbg.cspace) {
        for (int k = t; k < h * w; k += g.n) dbg.cspace[(size_t)n * h * w + k] = b_test(S.freeb[k / w], k % w) ? 1 : 0;
    }
    if (nsrc > 0) {
        snap_sources(sh, S, nsrc, g);
        if (t == 0) STAMP_NB(48);
        sssp_init_sources(sh, dist, nsrc, g);
    }
    // every read of the cspace scratch is done (snap_sources ended with a group sync): the render
    // group may now overwrite it with its raster tile -- zeroed here first when early_tile
    if (zero_tile) {
        uint4 *tz = reinterpret_cast<uint4 *>(&S);
        for (int k = t; k < SCRATCH_Q; k += g.n) tz[k] = uint4{0u, 0u, 0u, 0u};  // the rest: render params
        g.sync();
    }
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __hip_atomic_store(&sh.scratch_free, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        STAMP_NB(3);
    }
    if (nsrc == 0) return;
    sssp_rounds(sh, dist, nsrc, g);
    // the receptacle source's converged array -> its map slot's cache record (source 0 = the
    // receptacle when use_shortest_path_to_receptacle_map; envs.py:2071-2113 order)
    char *rec = dbg.rec_cache && cfg.use_shortest_path_to_receptacle_map
                    ? reinterpret_cast<char *>(dbg.rec_cache) + (size_t)ag.map_slot * rec_cache_bytes(h, w)
                    : nullptr;
    if (nsrc == 2 && G == 512 && !dbg.dist) {
        // each source's four waves take its maximum as soon as its own rounds end (the arrays are
        // independent), overlapping the other source's remaining rounds
        const int s = t >> 8;
        if (rec && s == 0) rec_export(rec, dist, h, w, sh.src_ok[0], nullptr, t & 255, 256);
        const float m = max_finite_part(dist + s * DIST_FLOATS, (h + 2) * sssp_pitch(w), t & 255, 256);
        if ((t & 63) == 0) sh.red[s][(t >> 6) & 3] = m;
        g.sync();
        if (t == 0) STAMP_NB(49);
        sssp_max_final(sh, nsrc, 4, (float)cfg.shortest_path_map_scale, t);
        if (t == 0) STAMP_NB(50);
        return;
    }
    g.sync();  // each source ran its own rounds: both arrays are final only now
    if (rec) rec_export(rec, dist, h, w, sh.src_ok[0], nullptr, t, g.n);
    if (t == 0) STAMP_NB(49);
    if (dbg.dist) {  // debug: the raw distances (unreachable -> +inf, read as sh.unreach like -inf)
        sssp_finish(sh, dist, nsrc, g);
        dump_dist(sh, dist, dbg.dist + (size_t)n * 2 * h * w, g);
        g.sync();
        if (t < nsrc) sh.unreach[t] = (sh.dmax[t] / 96.0f) * (float)cfg.shortest_path_map_scale;
    } else {
        sssp_max(sh, dist, nsrc, (float)cfg.shortest_path_map_scale, g);  // while the render waves finish
    }
    if (t == 0) STAMP_NB(50);
}

#ifndef SIMAPS_DEVICE_ONLY  // (simaps_mixed.hip includes this file for its device helpers only)
#ifdef SIMAPS_VGPR_CAP  // timing-only A/B build (tools/coresidency_model.py): the kernel squeezed to 8 waves
                        // per SIMD (<= 64 VGPRs, spills included) -- what two co-resident 16-wave stacks per
                        // CU would need; its LDS is dynamic so that the occupancy target is honoured
#define SIMAPS_GS_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
#else
#define SIMAPS_GS_ATTR
#endif
__global__ void __launch_bounds__(NT) SIMAPS_GS_ATTR get_state_kernel(
    simaps_config cfg, Geometry geo, const simaps_agent *__restrict__ agents, const simaps_env *__restrict__ envs,
    const simaps_robot *__restrict__ robots, const double *__restrict__ paths, const uint8_t *__restrict__ occupancy,
    const float *__restrict__ overhead, float *__restrict__ state, int C, simaps_debug dbg, unsigned *fault)
{
#define GS_MIXED 0
#include "get_state_body.inc"
#undef GS_MIXED
}
#endif

// ------------------------------------------------------------------------------------------------
// Reward lookups from the receptacle distance cache (simaps_sp_lookup)
// ------------------------------------------------------------------------------------------------
// Mapper.distance_to_receptacle (envs.py:2190-2194) between two map updates is answered by the
// reference from its GridGraph cache (shortest_paths.pyx:116-119, 156-163), which get_state filled
// with the receptacle-source SPFA: here the slot's cached array.  Per agent, one lane per target: a
// target pixel inside the rect whose cached value is above -inf is free = its own snapped cell
// (EDT distance 0, the common case) and reads its value; the others need the EDT snap, whose free
// bits are rebuilt from the cached array once per agent (only if some target needs them) and which
// runs two targets at a time (snap_sources).  Same values as sp_distance_kernel, bitwise.
struct LookupHdr {
    int h, w, i0, j0;
    int src_q[2][2], src_s[2][2], src_ok[2];
};
struct LookupScratch {
    B128 freeb[MAX_ROWS];
};
constexpr int LNT = 128;  // two waves: snap_sources' two slots
#ifndef SIMAPS_DEVICE_ONLY
__global__ void __launch_bounds__(LNT) sp_lookup_kernel(simaps_config cfg, const simaps_agent *__restrict__ agents,
                                                        const char *__restrict__ rec_cache, int rec_bytes,
                                                        const double *__restrict__ targets, int Q,
                                                        double *__restrict__ out)
{
    __shared__ LookupHdr sh;
    __shared__ LookupScratch S;
    __shared__ uint64_t slow_mask;
    const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int H = cfg.H, W = cfg.W, h = cfg.room_h, w = cfg.room_w, i0 = cfg.room_i0, j0 = cfg.room_j0;
    const int pw = sssp_pitch(w);
    const simaps_agent ag = agents[n];
    const char *rec = rec_cache + (size_t)ag.map_slot * rec_bytes;
    const int src_ok = reinterpret_cast<const int *>(rec)[1];
    const float *D = reinterpret_cast<const float *>(rec + REC_HDR);
    if (tid == 0) {
        sh.h = h;
        sh.w = w;
        sh.i0 = i0;
        sh.j0 = j0;
    }
    // dists[target] (pyx:156-163) as a Python float / 96; unreachable -> -1 (pyx:110-112)
    auto lookup = [&](int si, int sj) {
        float d = -1.0f;
        if (src_ok) {
            const float v = D[(si - i0 + 1) * pw + (sj - j0 + 1)];
            if (fabsf(v) != INFINITY) d = v;
        }
        return (double)d / PPM;
    };
    bool built = false;  // the free bits (uniform)
    for (int c0 = 0; c0 < Q; c0 += 64) {
        const int cn = Q - c0 < 64 ? Q - c0 : 64;
        if (tid < 64) {
            bool slow = false;
            if (tid < cn) {
                const double *t = targets + 2 * ((size_t)n * Q + c0 + tid);
                int qi, qj;
                pos_to_pix(t[0], t[1], H, W, qi, qj);
                const int qr = qi - i0, qc = qj - j0;
                const bool in = qr >= 0 && qr < h && qc >= 0 && qc < w;
                if (in && D[(qr + 1) * pw + qc + 1] != -INFINITY)
                    out[(size_t)n * Q + c0 + tid] = lookup(qi, qj);
                else
                    slow = true;
            }
            const uint64_t m = __ballot(slow);
            if (tid == 0) slow_mask = m;
        }
        lds_barrier();
        const uint64_t sm = slow_mask;
        if (sm && !built) {  // free bits of the rect rows, lane l -> columns l and l + 64
            for (int r = tid >> 6; r < h; r += LNT / 64) {
                const float *row = D + (r + 1) * pw + 1;
                const uint64_t lo = __ballot(lane < w && row[lane] != -INFINITY);
                const uint64_t hi = __ballot(lane + 64 < w && row[lane + 64] != -INFINITY);
                if (lane == 0) S.freeb[r] = B128{lo, hi};
            }
            built = true;
            lds_barrier();
        }
        for (uint64_t m = sm; m;) {
            int q[2] = {0, 0}, nq = 0;
            while (m && nq < 2) {
                q[nq++] = c0 + __builtin_ctzll(m);
                m &= m - 1;
            }
            if (tid < nq) {
                const double *t = targets + 2 * ((size_t)n * Q + q[tid]);
                pos_to_pix(t[0], t[1], H, W, sh.src_q[tid][0], sh.src_q[tid][1]);
            }
            lds_barrier();
            snap_sources(sh, S, nq, Group{tid, LNT, nullptr, LNT / 64});
            if (tid < nq) out[(size_t)n * Q + q[tid]] = sh.src_ok[tid] ? lookup(sh.src_s[tid][0], sh.src_s[tid][1]) : -1.0 / PPM;
            lds_barrier();
        }
        if (c0 + 64 < Q) lds_barrier();  // every wave has read slow_mask before the next chunk rewrites it
    }
}
#endif

// ------------------------------------------------------------------------------------------------
// GridGraph.shortest_path_image for arbitrary grids (one workgroup per grid)
// ------------------------------------------------------------------------------------------------
#ifndef SIMAPS_DEVICE_ONLY
__global__ void __launch_bounds__(NT) sssp_grid_kernel(int H, int W, const uint8_t *__restrict__ grids,
                                                      const int32_t *__restrict__ sources, float *__restrict__ out,
                                                      int wi0, int wj0, int wh, int ww, unsigned *fault)
{
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    Shared &sh = *reinterpret_cast<Shared *>(smem);
    float *dist = reinterpret_cast<float *>(smem + OFF_DIST);
    SsspScratch &S = *reinterpret_cast<SsspScratch *>(smem + OFF_UNION);
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint8_t *grid = grids + (size_t)b * H * W;
    if (tid == 0) {
        sh.h = wh; sh.w = ww; sh.i0 = wi0; sh.j0 = wj0;
        const int si = sources[2 * b], sj = sources[2 * b + 1];
        const bool ok = si >= wi0 && si < wi0 + wh && sj >= wj0 && sj < wj0 + ww && grid[(size_t)si * W + sj] != 0;
        sh.src_s[0][0] = si; sh.src_s[0][1] = sj; sh.src_ok[0] = ok;
    }
    const int nwords = (ww + 63) >> 6;
    for (int item = wave; item < wh * 2; item += NT / 64) {
        const int rr = item >> 1, wd = item & 1, c = wd * 64 + lane;
        const bool f = wd < nwords && c < ww && grid[(size_t)(wi0 + rr) * W + wj0 + c] != 0;
        const uint64_t m = __ballot(f);
        if (lane == 0) { if (wd == 0) S.freeb[rr].lo = m; else S.freeb[rr].hi = m; }
    }
    lds_barrier();
    sssp(sh, S, dist, 1);
    if (tid == 0) post_faults(fault, group_faults(sh.bar, sh.rounds, 1));
    // A blocked source has no edges but still dist 0 (pyx:84-88 set dists[source] before the loop).
    const int src_k = sh.src_s[0][0] * W + sh.src_s[0][1];
    for (int k = tid; k < H * W; k += NT) {
        const int i = k / W - wi0, j = k % W - wj0;
        float v = k == src_k ? 0.0f : -1.0f;
        if (i >= 0 && i < wh && j >= 0 && j < ww) {
            const float d = dist[(i + 1) * sssp_pitch(ww) + j + 1];
            if (d != __int_as_float(INF_BITS)) v = d;
        }
        out[(size_t)b * H * W + k] = v;
    }
}
#endif

// The robot class of agent ag with get_state_kernel's descriptor clamps (num_robots in [1,
// SIMAPS_MAX_ROBOTS], robot index < num_robots, class < 4); `bad` = something was clamped
// (SIMAPS_FAULT_DESCRIPTOR).
__device__ __forceinline__ int agent_robot_type(const simaps_agent &ag, const simaps_env *envs, const simaps_robot *robots,
                                                bool &bad)
{
    const simaps_env ev = envs[ag.env];
    bad = (unsigned)(ev.num_robots - 1) >= (unsigned)SIMAPS_MAX_ROBOTS || (unsigned)ag.robot >= (unsigned)ev.num_robots;
    const int nr = min(max(ev.num_robots, 1), SIMAPS_MAX_ROBOTS);
    const int r = (unsigned)ag.robot < (unsigned)nr ? ag.robot : 0;
    int type = robots[ev.robot_off + r].type;
    if ((unsigned)type > 3u) { bad = true; type = 0; }
    return type;
}

// ------------------------------------------------------------------------------------------------
// Reward lookups: OccupancyMap.shortest_path_distance (envs.py:2507-2512) from one source position to
// Q target positions on each agent's own map (Mapper.distance_to_receptacle, envs.py:2190-2194)
// ------------------------------------------------------------------------------------------------
#ifndef SIMAPS_DEVICE_ONLY
__global__ void __launch_bounds__(NT) sp_distance_kernel(simaps_config cfg, Geometry geo,
                                                         const simaps_agent *__restrict__ agents,
                                                         const simaps_env *__restrict__ envs,
                                                         const simaps_robot *__restrict__ robots,
                                                         const uint8_t *__restrict__ occupancy,
                                                         const double *__restrict__ sources,
                                                         const double *__restrict__ targets, int Q,
                                                         double *__restrict__ out, char *rec_cache, unsigned *fault)
{
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    Shared &sh = *reinterpret_cast<Shared *>(smem);
    float *dist = reinterpret_cast<float *>(smem + OFF_DIST);
    SsspScratch &S = *reinterpret_cast<SsspScratch *>(smem + OFF_UNION);
    const int n = blockIdx.x, tid = threadIdx.x;
    const int H = cfg.H, W = cfg.W;
    const simaps_agent ag = agents[n];
    OccLoad<NT> occ_regs;
    cspace_load<NT>(occ_regs, occupancy + (size_t)ag.map_slot * H * W, H, W, cfg.room_i0, cfg.room_j0, cfg.room_h,
                    cfg.room_w, tid);
    if (tid == 0) {
        bool bad;
        const int type = agent_robot_type(ag, envs, robots, bad);
        sh.flag[1] = bad;
        sh.h = cfg.room_h;
        sh.w = cfg.room_w;
        sh.i0 = cfg.room_i0;
        sh.j0 = cfg.room_j0;
        sh.r = geo.cspace_r[type];
        pos_to_pix(sources[2 * n], sources[2 * n + 1], H, W, sh.src_q[0][0], sh.src_q[0][1]);
        sh.nsrc = 1;
    }
    lds_barrier();
    build_cspace<NT>(S, &occ_regs, sh.h, sh.w, sh.r, whole_wg());
    snap_sources(sh, S, 1, whole_wg());
    const bool src_ok = sh.src_ok[0];
    sssp(sh, S, dist, 1);  // the source's distance image (GridGraph._spfa_with_cache, pyx:116-119)
    if (tid == 0) post_faults(fault, group_faults(sh.bar, sh.rounds, 1) | (sh.flag[1] ? SIMAPS_FAULT_DESCRIPTOR : 0u));
    if (rec_cache)  // the source is the receptacle (the caller's contract): keep the array for simaps_sp_lookup
        rec_export(rec_cache + (size_t)ag.map_slot * rec_cache_bytes(sh.h, sh.w), dist, sh.h, sh.w, src_ok, S.freeb, tid, NT);
    const int pw = sssp_pitch(sh.w);
    // dists[target] (pyx:156-163) as a Python float / LOCAL_MAP_PIXELS_PER_METER; unreachable -> -1
    // (pyx:110-112)
    auto lookup = [&](int si, int sj) {
        float d = -1.0f;
        if (src_ok) {
            const float v = dist[(si - sh.i0 + 1) * pw + (sj - sh.j0 + 1)];
            if (v != INFINITY) d = v;
        }
        return (double)d / PPM;
    };
    uint64_t &slow_mask = sh.dirty[0][0][0];  // (the SSSP's dirty masks are free now)
    for (int c0 = 0; c0 < Q; c0 += 64) {
        // wave 0, one lane per target: a free target pixel is its own snapped cell (EDT distance 0)
        const int cn = Q - c0 < 64 ? Q - c0 : 64;
        if (tid < 64) {
            bool slow = false;
            if (tid < cn) {
                const double *t = targets + 2 * ((size_t)n * Q + c0 + tid);
                int qi, qj;
                pos_to_pix(t[0], t[1], H, W, qi, qj);
                const int qr = qi - sh.i0, qc = qj - sh.j0;
                if (qr >= 0 && qr < sh.h && qc >= 0 && qc < sh.w && b_test(S.freeb[qr], qc))
                    out[(size_t)n * Q + c0 + tid] = lookup(qi, qj);
                else
                    slow = true;
            }
            const uint64_t m = __ballot(slow);
            if (tid == 0) slow_mask = m;
        }
        lds_barrier();
        // the others through the EDT feature transform, two at a time (snap_sources' slots)
        for (uint64_t m = slow_mask; m;) {
            int q[2] = {0, 0}, nq = 0;
            while (m && nq < 2) {
                q[nq++] = c0 + __builtin_ctzll(m);
                m &= m - 1;
            }
            if (tid < nq) {
                const double *t = targets + 2 * ((size_t)n * Q + q[tid]);
                pos_to_pix(t[0], t[1], H, W, sh.src_q[tid][0], sh.src_q[tid][1]);
            }
            lds_barrier();
            snap_sources(sh, S, nq, whole_wg());
            if (tid < nq) out[(size_t)n * Q + q[tid]] = sh.src_ok[tid] ? lookup(sh.src_s[tid][0], sh.src_s[tid][1]) : -1.0 / PPM;
            lds_barrier();
        }
        if (c0 + 64 < Q) lds_barrier();  // every wave has read slow_mask before the next chunk rewrites it
    }
}
#endif

// ------------------------------------------------------------------------------------------------
// Movement paths: OccupancyMap.shortest_path (envs.py:2478-2505) = straight-line test on cspace_thin,
// EDT snap, GridGraph.shortest_path (pyx:121-154): SPFA parents, approximate_polygon, pruning.
// ------------------------------------------------------------------------------------------------
// skimage.draw.line pixel t of (r0, c0) -> (r1, c1): closed-form Bresenham, last pixel = end point
__device__ __forceinline__ void line_pixel(int r0, int c0, int r1, int c1, int t, int &pr, int &pc)
{
    const int dr = abs(r1 - r0), dc = abs(c1 - c0), n = (dr > dc ? dr : dc) + 1;
    if (t == n - 1) { pr = r1; pc = c1; return; }
    const bool steep = dr > dc;
    const int major = steep ? dr : dc, minor = steep ? dc : dr;
    const int smaj = steep ? (r1 - r0 > 0 ? 1 : -1) : (c1 - c0 > 0 ? 1 : -1);
    const int smin = steep ? (c1 - c0 > 0 ? 1 : -1) : (r1 - r0 > 0 ? 1 : -1);
    const int kt = major > 0 ? (2 * minor * t + major) / (2 * major) : 0;
    if (steep) { pr = r0 + smaj * t; pc = c0 + smin * kt; }
    else { pc = c0 + smaj * t; pr = r0 + smin * kt; }
}

// cspace (the GridGraph grid): free iff inside the room rect and a free cspace bit
template <class SH>
__device__ __forceinline__ bool cs_free(const SH &sh, const SsspScratch &S, int i, int j)
{
    const int r = i - sh.i0, c = j - sh.j0;
    return r >= 0 && r < sh.h && c >= 0 && c < sh.w && b_test(S.freeb[r], c);
}

// cspace_thin = 1 - binary_dilation(min(room_mask, occupancy), disk(3)) (envs.py:2456): free iff no
// in-room occupied pixel within disk(3); S.win holds the occupancy window (rect + RMAX halo).
template <class SH>
__device__ __forceinline__ bool thin_free(const SH &sh, const SsspScratch &S, int i, int j)
{
    constexpr int R = 3;  // disk(ceil(HALF_WIDTH * 96)) (envs.py:2426)
    for (int dy = -R; dy <= R; dy++)
        for (int dx = -R; dx <= R; dx++) {
            if (dx * dx + dy * dy > R * R) continue;
            const int y = i + dy, x = j + dx;
            if (y < sh.i0 || y >= sh.i0 + sh.h || x < sh.j0 || x >= sh.j0 + sh.w) continue;  // room mask
            const int wr = y - (sh.i0 - RMAX), wc = x - (sh.j0 - RMAX);
            if ((S.win[wr][wc >> 6] >> (wc & 63)) & 1ull) return false;
        }
    return true;
}

// wave-parallel: is every pixel of line (r0, c0) -> (r1, c1) free (thin ? cspace_thin : cspace)?
// grid == 1 bits of a raw GridGraph grid (grid_path_kernel; kept in S.dtab[0], which the SPFA arrays
// do not overlay): the line-of-sight test of pyx:146 counts (1 - grid[rr, cc]) != 0 in uint8, i.e.
// any cell != 1
template <class SH>
__device__ __forceinline__ bool one_free(const SH &sh, const SsspScratch &S, int i, int j)
{
    const int r = i - sh.i0, c = j - sh.j0;
    return r >= 0 && r < sh.h && c >= 0 && c < sh.w && b_test(S.dtab[0][r], c);
}

enum LineMask { LINE_CSPACE = 0, LINE_THIN = 1, LINE_GRID_ONE = 2 };

template <class SH>
__device__ __forceinline__ bool line_free(const SH &sh, const SsspScratch &S, int r0, int c0, int r1, int c1, int mask)
{
    const int lane = threadIdx.x & 63;
    const int n = max(abs(r1 - r0), abs(c1 - c0)) + 1;
    bool blocked = false;
    for (int t = lane; t < n; t += 64) {
        int pr, pc;
        line_pixel(r0, c0, r1, c1, t, pr, pc);
        blocked |= mask == LINE_THIN ? !thin_free(sh, S, pr, pc)
                   : mask == LINE_GRID_ONE ? !one_free(sh, S, pr, pc) : !cs_free(sh, S, pr, pc);
    }
    return __ballot(blocked) == 0;
}

// ------------------------------------------------------------------------------------------------
// Path kernels' LDS: one 256-thread workgroup per query, its LDS sized for the room so that several
// queries share a CU -- the exact SPFA is one wave's serial pop loop (latency-bound), so throughput
// comes from residency.  Layout (PathLds<CELLS>):
//   PathHdr                       query header (the Shared fields the snap / path steps read)
//   SsspScratch                   occupancy window, free bits, dilation table (build_cspace); after
//                                 the cspace is built only win (straight-line test), freeb and dtab[0]
//                                 (grid == 1 bits of grid paths) stay live, and
//   arrays at dtab[1]:            dist   f32 [CELLS]   SPFA distances (free: inf, blocked / border -inf)
//                                 queue  u16 [CELLS]   ring of cell indices (live entries <= cells)
//                                 pin    u8  [CELLS]   bits 0-3: 1 + direction of the parent edge (0: none),
//                                                      bit 4: in queue
// 7 B per cell: small rooms (46 x 95 cells) take 39 KB -> 4 queries per CU; rooms up to the
// SIMAPS_MAX_ROOM_CELLS limit 70 KB -> 2 per CU.  (The round-2 kernels used the 158 KB get_state
// layout, one 1024-thread query per CU.)
// ------------------------------------------------------------------------------------------------
#ifndef SIMAPS_POP_CAP  // the diagnostic build (tests/test_gpu_faults.py) lowers it to exercise the fault path
#define SIMAPS_POP_CAP (1 << 24)
#endif
#ifndef SIMAPS_SPFA_PIPE  // the round-4 software-pipelined pop (0: the round-3 pop, for A/B builds)
#define SIMAPS_SPFA_PIPE 1
#endif
#ifndef SIMAPS_SPFA_RING  // > 0: the diagnostic ring build (tests/test_gpu_faults.py) -- a queue ring of at most
#define SIMAPS_SPFA_RING 0  // this many slots, so that the ring wraps many times per query (the product's
#endif                      // ring has one slot per cell and rarely wraps); a live queue past it is a fault
constexpr int PNT = 256;  // path workgroup: 4 waves (build_cspace needs >= 4 for its row blocks)
constexpr int PATH_SMALL_CELLS = 4608;  // >= (44 + 2) * 95: every small_* room
struct PathHdr {
    int h, w, i0, j0, r, nsrc;
    int src_q[2][2], src_s[2][2], src_ok[2];
    int flag[2];
    int nseg;
    unsigned fault;        // SIMAPS_FAULT_* bits of this query
    int changed[3];        // (EARLY) per-round "a sweep improved a cell" flags
    uint64_t dirty[4][2];  // (EARLY) per sweep direction: lines to relax again
    float finT;            // (EARLY) the target's fixpoint distance
    unsigned trio[4];      // (OVL) the sweep waves' Group barrier (arrivals, generation, timeout flag)
    int swept;             // (OVL) 1 once the fixpoint (and finT) is complete: released by the sweep waves
};
constexpr int OFF_PS = align16((int)sizeof(PathHdr));
constexpr int OFF_PA = OFF_PS + align16((int)(offsetof(SsspScratch, dtab) + sizeof(B128) * MAX_WIN_ROWS));
// (The early-exit variant's SSSP fixpoint runs in the dist array and is then parked in global memory --
// the per-stream scratch of path_scratch(), CELLS f32 per query -- so both variants have this layout.
// The overlapped variant, OVL, keeps the fixpoint in its own LDS array `fix` [CELLS] f32 after pin:
// its sweeps run on waves 1-3 while wave 0 already pops, so the two arrays live side by side.)
template <int CELLS, bool OVL = false>
constexpr int path_lds_bytes()
{
    return align16(OFF_PA + align16(7 * CELLS) + (OVL ? 4 * CELLS : 0) > OFF_PS + (int)sizeof(SsspScratch)
                       ? OFF_PA + align16(7 * CELLS) + (OVL ? 4 * CELLS : 0)
                       : OFF_PS + (int)sizeof(SsspScratch));
}
static_assert(path_lds_bytes<PATH_SMALL_CELLS>() * 4 <= 160 * 1024, "4 small-room queries per CU");
static_assert(path_lds_bytes<SIMAPS_MAX_ROOM_CELLS>() * 2 <= 160 * 1024, "2 queries per CU at the room limit");
static_assert(path_lds_bytes<PATH_SMALL_CELLS, true>() * 2 <= 160 * 1024, "OVL: 2 small-room queries per CU");
static_assert(path_lds_bytes<SIMAPS_MAX_ROOM_CELLS, true>() <= 160 * 1024, "OVL: 1 query per CU at the room limit");
// per-CU residency of a path kernel (LDS decides it: 4 waves of <= 128 VGPRs fit many times over)
template <int CELLS, bool OVL>
constexpr int path_per_cu() { return (160 * 1024) / path_lds_bytes<CELLS, OVL>(); }
static_assert(MAX_ROWS <= 256 && SIMAPS_MAX_ROOM_W <= 256, "rect cells pack as (row << 8) | col");

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

// pyx:30 direction order [0,-1],[0,1],[-1,-1],[-1,0],[-1,1],[1,-1],[1,0],[1,1]: cell offset of edge k
__device__ __forceinline__ int dir_off(int k, int pw)
{
    const int di = k < 2 ? 0 : (k < 5 ? -1 : 1);
    const int dj = k < 2 ? (k == 0 ? -1 : 1) : ((k - 2) % 3) - 1;
    return di * pw + dj;
}

#ifndef SIMAPS_SPFA_ASM  // the common pops as one inline-asm loop (0: the C++ pop alone, for A/B builds)
#define SIMAPS_SPFA_ASM 1
#endif
// The common SPFA pop (shortest_paths.pyx:89-107) as one inline-asm loop (round 4).  The C++ pop in
// path_core costs ~85 instructions with the compiler's exec juggling and register copies; this one
// ~43 (two pops per iteration, so the next second needs no copy).  The next pop's LDS reads are
// issued right after this pop's writes, so their latency overlaps
// the bookkeeping and the next pop's checks; the improved heads and u's own pin byte go out as one
// write per array (lane 8 -- doff 0, the popped vertex -- rewrites its unchanged distance), not as a
// same-address write from every lane.  The loop runs pops while each is "common": the queue keeps
// >= 3 entries after the pop, no pushed distance is below the front's (no SLF swap, pyx:104-107),
// the pop does not lower the front's distance, and neither the tail nor the read-ahead slot reaches
// the ring's end (no slot wraps).  Then the pushes go to the tail in edge order, slot = tail + rank
// among the pushed edges, and the next front / second are the current second / third.  It returns
// when its budget runs out (`left`, or the wrap / count limits), when the early-exit mode's 32-pop
// target check (done in the loop while tchk is set) finds the target final, or when the pop at hand
// is not common -- before any of that pop's writes,
// with its reads (vv / dv / pv / dF0 / pth, issued one pop ahead, as path_core's pf_* values)
// complete -- so that the C++ pop replays that one exactly.  State as in path_core: u the front, F0
// the second, qn the slot of F0, qt the tail slot, cnt the live entries including u.  DIST / QUEUE /
// PIN: the byte offsets of the LDS arrays (checked by the caller).  (Round 5 tried lane 8's write
// values without the two selects -- weight 0 on lane 8 and one v_and_or -- and measured it 3 %
// slower per pop: profiles/r5i_*.)
// Wait states: a VALU SGPR write is read by a VALU >= 2 instructions later (du); the opening s_nop
// covers the compiler's last writes of the inputs.  The wave's LDS operations complete in order, so
// one lgkmcnt(0) before each pop waits for the read-ahead and everything before it.
template <int DIST, int QUEUE, int PIN>
__device__ __forceinline__ void spfa_fast_pops(int &u, int &F0, int &qn, int &qt, int &cnt, int &left, int &lim_add,
                                               int ring, int &vv, float &dv, int &pv, float &dF0, int &pth, int doff,
                                               float wl, int pbits, int tchk, int tv, float finT)
{
    static_assert(PIN + 255 < 65536 && QUEUE + 4 < 65536, "ds offsets are 16-bit");
    const uint64_t l8 = 1ull << 8;  // lane 8: the popped vertex itself (doff 0)
    // Pops the loop may run with no per-pop test but its budget: no ring wrap (the tail grows by <= 8
    // per pop and stays within ring - 8, the read-ahead slot by 1 and stays within ring - 3), >= 4
    // live entries before every pop (the count drops by <= 1 per pop: budget cnt - 3) and at most
    // `left`.  qn grows by exactly 1 per pop and u is lane 8's edge head of the read-ahead, so
    // neither is carried; with no wrap the live entries are cnt = qt - qn + 1.
    // The budget is run in segments of min(left, what remains of it) pops.  When a segment ends at
    // `left` = 0 and tchk is set (the early-exit mode, target not yet at its fixpoint distance), the
    // loop itself makes path_core's 32-pop check -- one LDS read of the target's distance -- and
    // either returns (the target is final: path_core walks its chain) or runs the next 32 pops
    // (lim_add counts those, so path_core's pop accounting `pops = lim - left` still holds).
    int gb = __builtin_amdgcn_readfirstlane(min(cnt - 3, min((ring - 8 - qt) >> 3, ring - 3 - qn)));
    const int gb0 = gb;
    int seg = __builtin_amdgcn_readfirstlane(min(left, gb)), bud = seg, lft = __builtin_amdgcn_readfirstlane(left), ladd = 0;
    // the target's byte offset in the distance array, or -1: no target checks in the loop
    const int tv4 = __builtin_amdgcn_readfirstlane(tchk ? 4 * tv : -1);
    const uint32_t fin = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(finT));
    uint64_t ex, nq, fm, im, sw;
    int du, th, t;
    float nd;
    int ta, tb, tc, td;
    if (seg > 0 && qt >= qn) {  // (qt < qn: the live entries wrap the ring; the C++ pop runs)
        int tq = 2 * qn;  // byte offset of slot qn in the queue (the read-ahead slot is qn + 2)
        // two pops per iteration with the second's registers swapped (no copy of the next second into
        // F0, one branch and one read-ahead slot increment per two pops)
#define FP_POP(A, B, QOFF, L9, L8, LS)                                                              \
            "v_readlane_b32 %[du], %[dv], 8\n\t"                                                   \
            "v_readfirstlane_b32 " B ", %[pth]\n\t"                                                \
            "v_cmp_gt_u32_e64 %[nq], 16, %[pv]\n\t"                                                \
            "v_and_b32_e32 %[tb], 15, %[pv]\n\t"                                                   \
            "v_add_f32_e32 %[nd], %[du], %[wl]\n\t"                                                \
            "v_cmp_eq_u32_e64 %[fm], " A ", %[vv]\n\t"                                             \
            "v_cmp_lt_f32_e64 %[im], %[nd], %[dv]\n\t"                                             \
            "v_cmp_lt_f32_e64 %[sw], %[nd], %[dF0]\n\t"                                            \
            "v_cndmask_b32_e64 %[tb], %[pbits], %[tb], %[l8]\n\t"                                  \
            "v_cndmask_b32_e64 %[td], %[nd], %[dv], %[l8]\n\t"                                     \
            "v_lshlrev_b32_e32 %[ta], 2, %[vv]\n\t"                                                \
            "s_and_b64 %[nq], %[nq], %[im]\n\t"                                                    \
            "s_and_b64 %[fm], %[fm], %[im]\n\t"                                                    \
            "s_and_b64 %[sw], %[sw], %[nq]\n\t"                                                    \
            "s_or_b64 %[sw], %[sw], %[fm]\n\t"                                                     \
            "s_cmp_lg_u64 %[sw], 0\n\t"                                                            \
            "s_cbranch_scc1 " L9 "\n\t"                                                            \
            "s_or_b64 exec, %[im], %[l8]\n\t"                                                      \
            "ds_write_b32 %[ta], %[td] offset:%c[DIST]\n\t"                                        \
            "ds_write_b8 %[vv], %[tb] offset:%c[PIN]\n\t"                                          \
            "s_cmp_eq_u64 %[nq], 0\n\t"                                                            \
            "s_cbranch_scc1 " LS "f\n\t"                                                                 \
            "s_mov_b64 exec, %[nq]\n\t"                                                            \
            "s_mov_b64 vcc, %[nq]\n\t"                                                             \
            "v_mbcnt_lo_u32_b32 %[td], vcc_lo, 0\n\t"                                              \
            "v_add_u32_e32 %[td], %[qt], %[td]\n\t"                                                \
            "v_lshlrev_b32_e32 %[td], 1, %[td]\n\t"                                                \
            "ds_write_b16 %[td], %[vv] offset:%c[QUEUE]\n"                                         \
            LS ":\n\t"                                                                             \
            "s_mov_b64 exec, %[ex]\n\t"                                                            \
            "v_add_u32_e32 %[vv], " A ", %[doff]\n\t"                                              \
            "v_lshlrev_b32_e32 %[tb], 2, %[pth]\n\t"                                               \
            "v_lshlrev_b32_e32 %[ta], 2, %[vv]\n\t"                                                \
            "ds_read_b32 %[dF0], %[tb] offset:%c[DIST]\n\t"                                        \
            "ds_read_u16 %[pth], %[tc] offset:%c[" QOFF "]\n\t"                                    \
            "ds_read_b32 %[dv], %[ta] offset:%c[DIST]\n\t"                                         \
            "ds_read_u8 %[pv], %[vv] offset:%c[PIN]\n\t"                                           \
            "s_bcnt1_i32_b64 %[t], %[nq]\n\t"                                                      \
            "s_add_u32 %[qt], %[qt], %[t]\n\t"                                                     \
            "s_sub_u32 %[bud], %[bud], 1\n\t"                                                      \
            "s_cmp_le_i32 %[bud], 0\n\t"                                                           \
            "s_cbranch_scc1 " L8 "\n\t"                                                            \
            "s_waitcnt lgkmcnt(0)\n\t"
        // At a segment's end (its last pop's reads issued): account the segment, wait for the reads, and
        // leave unless it ended at `left` = 0 with target checks on; then check the target (leave if
        // it is final) and run the next 32 pops after FIX (the register fix-up for the iteration half).
#define FP_REFILL(FIX, LEXIT)                                                                      \
            "s_sub_u32 %[gb], %[gb], %[seg]\n\t"                                                   \
            "s_sub_u32 %[lft], %[lft], %[seg]\n\t"                                                 \
            "s_mov_b32 %[seg], 0\n\t"                                                             \
            "s_waitcnt lgkmcnt(0)\n\t"                                                             \
            "s_cmp_le_i32 %[gb], 0\n\t"                                                            \
            "s_cbranch_scc1 " LEXIT "\n\t"                                                         \
            "s_cmp_eq_u32 %[tv4], -1\n\t"                                                          \
            "s_cbranch_scc1 " LEXIT "\n\t"                                                         \
            "s_cmp_gt_i32 %[lft], 0\n\t"                                                           \
            "s_cbranch_scc1 " LEXIT "\n\t"                                                         \
            "v_mov_b32_e32 %[ta], %[tv4]\n\t"                                                      \
            "ds_read_b32 %[td], %[ta] offset:%c[DIST]\n\t"                                         \
            "s_waitcnt lgkmcnt(0)\n\t"                                                             \
            "v_readfirstlane_b32 %[t], %[td]\n\t"                                                  \
            "s_cmp_eq_u32 %[t], %[fin]\n\t"                                                        \
            "s_cbranch_scc1 " LEXIT "\n\t"                                                         \
            "s_add_u32 %[ladd], %[ladd], 32\n\t"                                                   \
            "s_mov_b32 %[lft], 32\n\t"                                                             \
            "s_min_u32 %[seg], %[gb], 32\n\t"                                                      \
            "s_mov_b32 %[bud], %[seg]\n\t"                                                         \
            FIX                                                                                    \
            "s_branch 1b\n"
        asm volatile(
            "s_nop 1\n\t"
            "s_mov_b64 %[ex], exec\n\t"
            "v_mov_b32_e32 %[tc], %[tq]\n"
            "1:\n\t"
            FP_POP("%[F0]", "%[th]", "QUEUE4", "9f", "8f", "31")
            FP_POP("%[th]", "%[F0]", "QUEUE6", "7f", "6f", "32")
            "v_add_u32_e32 %[tc], 4, %[tc]\n\t"
            "s_branch 1b\n"
            // a segment ended in the first pop of an iteration (the next second is in th)
            "8:\n\t"
            FP_REFILL("s_mov_b32 %[F0], %[th]\n\tv_add_u32_e32 %[tc], 2, %[tc]\n\t", "5f")
            "5:\n\t"
            "s_mov_b32 %[F0], %[th]\n\t"
            "s_branch 9f\n"
            // an uncommon pop in the second pop of an iteration (its second is in th)
            "7:\n\t"
            "s_mov_b32 %[F0], %[th]\n\t"
            "s_branch 9f\n"
            // a segment ended in the second pop of an iteration
            "6:\n\t"
            FP_REFILL("v_add_u32_e32 %[tc], 4, %[tc]\n\t", "9f")
            "9:\n\t"
            : [F0] "+s"(F0), [qt] "+s"(qt), [bud] "+s"(bud), [seg] "+s"(seg), [gb] "+s"(gb), [lft] "+s"(lft),
              [ladd] "+s"(ladd),
              [vv] "+v"(vv), [dv] "+v"(dv), [pv] "+v"(pv), [dF0] "+v"(dF0), [pth] "+v"(pth),
              [ex] "=&s"(ex), [nq] "=&s"(nq), [fm] "=&s"(fm), [im] "=&s"(im), [sw] "=&s"(sw), [du] "=&s"(du),
              [th] "=&s"(th), [t] "=&s"(t), [nd] "=&v"(nd), [ta] "=&v"(ta), [tb] "=&v"(tb), [tc] "=&v"(tc),
              [td] "=&v"(td)
            : [tq] "s"(tq), [l8] "s"(l8), [tv4] "s"(tv4), [fin] "s"(fin), [doff] "v"(doff), [wl] "v"(wl), [pbits] "v"(pbits), [DIST] "i"(DIST),
              [QUEUE] "i"(QUEUE), [QUEUE4] "i"(QUEUE + 4), [QUEUE6] "i"(QUEUE + 6), [PIN] "i"(PIN)
            : "memory", "scc", "vcc");
#undef FP_POP
#undef FP_REFILL
        const int done = (gb0 - gb) + (seg - bud);  // pops run (the one at hand, if uncommon, is not among them)
        left = lft - (seg - bud);
        lim_add = ladd;
        qn += done;
        cnt = qt - qn + 1;
        u = __builtin_amdgcn_readlane(vv, 8);
    }
}

// Steps (3)-(6) of the movement path on the LDS-resident free bits (S.freeb) between the cells
// sh.src_s[0] (source) and sh.src_s[1] (target), both inside the window: the exact SPFA (run_spfa:
// the source is a free cell of the window; otherwise only the source is reached), the parent walk,
// approximate_polygon and the line-of-sight pruning on `line_mask`.  Leaves the kept waypoints in
// outp[0, cnt) (u16 rect cells (row << 8) | col, target first, i.e. before pyx:152's reversal) and
// returns cnt in wave 0.  All PNT threads call it.
//
// OVL (round 4, with EARLY): the sweeps and the SPFA overlap.  Waves 1-3 relax the fixpoint in their
// own LDS array `fix` (directions 0 / 1 / 2 then 3, rounds separated by the LDS barrier of a
// 3-wave Group) while wave 0 pops from the first cycle; wave 0 starts its target
// checks at the first 32-pop boundary after the sweep waves released `swept`.  Any schedule of exact
// relaxations reaches the same unique f32 fixpoint and the SPFA never reads `fix` before `swept`, so
// the results are those of EARLY; the fixpoint stays in LDS (no global scratch, no copy, chain checks
// read LDS), so the launch also runs under graph capture.
template <int CELLS, bool EARLY, bool OVL = false>
__device__ __forceinline__ int path_core(PathHdr &sh, SsspScratch &S, char *arr, int H, int W, bool run_spfa,
                                         int line_mask, float *gfin, const uint16_t *&outp_ret)
{
    float *dist = reinterpret_cast<float *>(arr);
    uint16_t *queue = reinterpret_cast<uint16_t *>(arr + 4 * CELLS);
    uint8_t *pin = reinterpret_cast<uint8_t *>(arr + 6 * CELLS);
    // after the parent walk: dense path (u16 rect cells) in the queue region, chain flags in pin,
    // the Douglas-Peucker stack (u16 pairs) in the dist region; then the sparse points and the kept
    // waypoints (u16 each) in the dist region
    uint16_t *dense = queue;
    uint32_t *stack = reinterpret_cast<uint32_t *>(arr);
    uint16_t *sparse = reinterpret_cast<uint16_t *>(arr), *outp = sparse + CELLS;
    uint8_t *chain = pin;
    outp_ret = outp;
    const int tid = threadIdx.x, lane = tid & 63;
    const int h = sh.h, w = sh.w, pw = sssp_pitch(w), cells = (h + 2) * pw;
    // (3) GridGraph._spfa (pyx:69-114) from the snapped source, exactly: one wave, the 8 out-edges of
    // a popped vertex evaluated by lanes 0..7 (distinct heads, so in parallel), then the pushes and
    // SLF swaps in edge order.  inf = 2 * H * W (pyx:38); queue as a ring (live entries <= cells).
    // Blocked and border cells hold -inf, so `new < dist[v]` is false for them: no free-bit test per
    // edge.  Per pop ONE round of LDS reads (dist[u], dist[v], pin[v] -- lane 8's v is u itself, so
    // its pin read is u's --, the next front) -- the front of the queue lives in a register (it is
    // either the prefetched next entry or the vertex an SLF swap just put there), so no read waits
    // for the previous pop's writes except the SLF front's distance, read only when a pop pushes.
    const float INFR = (float)(2 * H * W);
    static_assert(!OVL || EARLY, "OVL is a schedule of the early-exit variant");
    float *fix = OVL ? reinterpret_cast<float *>(arr + align16(7 * CELLS)) : nullptr;
    if (tid == 0) STAMP_NB(2);
    const int su = (sh.src_s[0][0] - sh.i0 + 1) * pw + (sh.src_s[0][1] - sh.j0 + 1);
    const int tv = (sh.src_s[1][0] - sh.i0 + 1) * pw + (sh.src_s[1][1] - sh.j0 + 1);
    for (int k = tid; k < cells; k += PNT) {
        const int rr = k / pw, cc = k - rr * pw;  // (once per cell)
        const bool fr = rr >= 1 && rr <= h && cc >= 1 && cc <= w && b_test(S.freeb[rr - 1], cc - 1);
        if (OVL) {  // the SPFA's initial state in dist, the sweeps' (source at 0) in fix
            dist[k] = fr ? INFR : -INFINITY;
            fix[k] = k == su ? 0.0f : (fr ? INFINITY : -INFINITY);
        } else {
            dist[k] = fr ? (EARLY ? INFINITY : INFR) : -INFINITY;  // (EARLY: the sweeps' initial state)
        }
        pin[k] = 0;
        queue[k] = 0;  // (every ring slot holds a cell index: the prefetched `second` needs no clamp)
    }
    if (EARLY && tid < 8) {  // only the source's row / column is dirty (all else is +-inf)
        const int d2 = tid >> 1, word = tid & 1;
        const int bit = d2 < 2 ? sh.src_s[0][0] - sh.i0 : sh.src_s[0][1] - sh.j0;
        sh.dirty[d2][word] = (bit >> 6) == word ? 1ull << (bit & 63) : 0ull;
        if (tid < 3) sh.changed[tid] = 0;
        if (tid == 3) sh.trio[0] = sh.trio[1] = sh.trio[2] = 0u, sh.swept = 0;
    }
    lds_barrier();
    if (OVL && run_spfa && tid >= 64) {
        // waves 1-3: the fixpoint in fix, directions 0 and 1 on waves 1 and 2, 2 then 3 on wave 3 (the
        // marks make any order exact); the 3-slot round flags as in the EARLY rounds below
        const int wave = tid >> 6;
        const Group g3{tid - 64, PNT - 64, sh.trio, PNT / 64 - 1};
        int steps = 0, round = 0;
        for (;; round++) {
            if (tid == 64) sh.changed[(round + 1) % 3] = 0;
            bool chg = sweep(fix, h, w, pw, wave == 3 ? 2 : wave - 1, sh.dirty, steps);
            if (wave == 3) chg = sweep(fix, h, w, pw, 3, sh.dirty, steps) || chg;
            if (chg && lane == 0) sh.changed[round % 3] = 1;
            g3.sync();
            if (!sh.changed[round % 3] || round >= h * w + 16) break;
        }
        if (tid == 64) {
            const unsigned f = (round >= h * w + 16 ? SIMAPS_FAULT_ROUNDS : 0u) | (sh.trio[2] ? SIMAPS_FAULT_TIMEOUT : 0u);
            if (f) fault_or(sh.fault, f);
            sh.finT = fix[tv];
            STAMP_VAL(8, round + 1);
            STAMP_NB(10);  // (stamp build: the sweeps' end)
            // (local-only fence, as Group::sync: an acquire / release atomic would also wait for global accesses)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __hip_atomic_store(&sh.swept, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (EARLY && !OVL && run_spfa) {
        // The f32 fixpoint of the graph from the source -- the SPFA's final distances, bitwise (SURVEY
        // a10) -- by the get_state sweeps, one direction per wave, rounds until nothing improves.
        // A vertex whose SPFA distance already equals it can never improve again, so its parent is
        // final: the SPFA below may stop as soon as the target's whole parent chain is final.  The
        // sweeps run in the dist array; the fixpoint then moves to this query's global scratch (read
        // back only along the parent chain) and dist takes the SPFA's initial state.
        if (tid == 0) dist[su] = 0.0f;
        lds_barrier();
        const int wave = tid >> 6;
        int steps = 0, round = 0;
        for (;; round++) {
            if (tid == 0) sh.changed[(round + 1) % 3] = 0;
            if (sweep(dist, h, w, pw, wave, sh.dirty, steps) && lane == 0 && !SSSP_CHECK) sh.changed[round % 3] = 1;
            lds_barrier();
            if (SSSP_CHECK) {
                if (sssp_check(dist, h, w, pw, sh.dirty, tid, PNT) && lane == 0) sh.changed[round % 3] = 1;
                lds_barrier();
            }
            if (!sh.changed[round % 3] || round >= h * w + 16) break;
        }
        if (tid == 0 && round >= h * w + 16) fault_or(sh.fault, SIMAPS_FAULT_ROUNDS);
        if (tid == 0) sh.finT = dist[tv];
        for (int k = tid; k < cells; k += PNT) {
            const float f = dist[k];
            gfin[k] = f;
            dist[k] = f == -INFINITY ? -INFINITY : INFR;
        }
        __syncthreads();  // (global stores of the other waves -> wave 0's chain checks; LDS likewise)
        if (tid == 0) STAMP_VAL(8, round + 1);
        if (tid == 0) STAMP_NB(10);  // (stamp build: the sweeps' end)
    }
    if (tid < 64 && run_spfa) {
        const int doff = lane < 8 ? dir_off(lane, pw) : 0;
        const float wl = (lane >= 2 && lane < 8 && lane != 3 && lane != 6) ? SQRT2F : 1.0f;
        const uint8_t pbits = (uint8_t)((lane + 1) | 0x10);  // a relaxed head: parent edge `lane`, queued
        if (lane == 0) { dist[su] = 0.0f; queue[0] = (uint16_t)su; pin[su] = 0x10; }
        __builtin_amdgcn_wave_barrier();
        // live entries queue[qh .. qt) (mod ring); front == queue[qh]; second == queue[qh + 1] when
        // count >= 2 (prefetched one pop ahead, so the SLF front's distance is read in the same round
        // as the popped vertex's edges instead of after them)
        // (front / second start from the uniform su as SGPR values: a VGPR start would make the
        // loop carry them in VGPRs, with a move and a readfirstlane each per pop)
        const int su_s = __builtin_amdgcn_readfirstlane(su);
        const int ring = SIMAPS_SPFA_RING > 0 && SIMAPS_SPFA_RING < cells ? SIMAPS_SPFA_RING : cells;
        // (qn: the slot after qh, carried so that a pop computes one ring wrap, not two)
        int qh = 0, qn = 1, qt = 1, count = 1, front = su_s, second = su_s;
        // (the wave's stores below are made by every lane with the same address and value: no exec
        // masking around them)
        lds_float *Ld = (lds_float *)dist;
        lds_u16 *Lq = (lds_u16 *)queue;
        lds_u8 *Li = (lds_u8 *)pin;
        // pops: done so far; lim: the next pop count at which the loop looks beyond its queue -- the
        // pop cap (never reached by a correct SPFA) or, in EARLY, the next early-exit check -- so the
        // common pop pays one scalar compare for both
        int pops = 0, gap = 64, lim = EARLY ? 32 : SIMAPS_POP_CAP;
        bool early = false, tfinal = false;
        // the target's fixpoint distance (uniform: kept in an SGPR); OVL: known once `swept` is seen
        bool have_fin = !OVL;
        float finT = EARLY && !OVL ? __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sh.finT))) : 0.0f;
        // an unreachable target (fixpoint +inf) never gets a parent: the SPFA cannot change the path
        // (likewise a blocked target, fixpoint -inf: grid paths; movement-path targets are snapped)
        if (EARLY && !OVL && (finT == INFINITY || finT == -INFINITY)) count = 0, early = true;
#if SIMAPS_SPFA_PIPE
        // the reads of the next pop, issued one pop ahead: its vertex's 8 edge heads and itself
        // (lane 8), the distance of the entry after it (the SLF front during that pop) and the slot
        // after that one
        int pf_v = 0, pf_pv = 0, pf_third = 0;
        float pf_dv = 0.0f, pf_dF0 = 0.0f;
        auto pf_issue = [&](int fr, int sc, int slot) {
            pf_v = fr + doff;
            pf_dv = Ld[pf_v];
            pf_pv = Li[pf_v];
            pf_dF0 = Ld[sc];
            pf_third = Lq[slot];
        };
        pf_issue(front, second, qn + 1 == ring ? 0 : qn + 1);
        // the asm pop addresses the LDS arrays by their compile-time offsets in the kernel's LDS block
        const bool asm_ok = (uint32_t)(uintptr_t)Ld == (uint32_t)OFF_PA && (uint32_t)(uintptr_t)Lq == (uint32_t)(OFF_PA + 4 * CELLS) &&
                            (uint32_t)(uintptr_t)Li == (uint32_t)(OFF_PA + 6 * CELLS);
#endif
        // pop rounds (inner loop: one exit, so the common pop ends in one compare) up to `lim`, then
        // (EARLY) an early-exit check
        if (count > 0)
            for (;;) {
                int left = lim - pops;  // pops of this round (the common pop's one exit test: min(count, left))
                for (;;) {
#if SIMAPS_SPFA_PIPE && SIMAPS_SPFA_ASM
                    if (asm_ok) {  // the common pops in one asm loop; it returns at `left` = 0 or an uncommon pop
                        int fs = __builtin_amdgcn_readfirstlane(front), ss = __builtin_amdgcn_readfirstlane(second);
                        int ladd = 0;
                        spfa_fast_pops<OFF_PA, OFF_PA + 4 * CELLS, OFF_PA + 6 * CELLS>(
                            fs, ss, qn, qt, count, left, ladd, ring, pf_v, pf_dv, pf_pv, pf_dF0, pf_third, doff, wl,
                            (int)pbits, __builtin_amdgcn_readfirstlane(EARLY && have_fin && !tfinal ? 1 : 0),
                            __builtin_amdgcn_readfirstlane(tv), finT);
                        lim += ladd;
                        front = fs;
                        second = ss;
                        if (left <= 0) break;
                    }
#endif
#if SIMAPS_SPFA_PIPE
                    {
                    // The pop, software-pipelined (round 4).  Its LDS reads -- the popped vertex's 8 edge
                    // heads and itself, the next front's distance, the slot after it -- were issued at the
                    // end of the previous pop, right after that pop's writes, so their latency overlaps
                    // that pop's queue bookkeeping.  The common pop (the SLF swap of pyx:104-107 happens in
                    // ~0.4 % of pops) is lane-parallel: with no pushed distance below the front's, the
                    // pushes go to the tail in edge order (slot = tail + rank among the pushed edges), so
                    // the next front is known (second) and its reads can be issued at once.  Every other
                    // pop -- a possible swap, the front lowered by this pop (its distance changes between
                    // edges), or a queue of <= 2 entries (the slots read ahead may be written by this
                    // pop's pushes) -- replays the pushes with an SALU loop over the edge bits in edge
                    // order, the front's distance in an SGPR.  Distances here are >= 0 or INFR (blocked
                    // cells hold -inf and are never relaxed or pushed), so float order is unsigned order
                    // and the SLF test is one s_cmp.  Masks are 32-bit: only lanes 0..7 carry edges.
                    const int u = __builtin_amdgcn_readfirstlane(front);
                    qh = qn;
                    count--;
                    const int F0 = __builtin_amdgcn_readfirstlane(second);
                    const int q2 = qh + 1 == ring ? 0 : qh + 1;
                    qn = q2;
                    const int v = pf_v;
                    const float dv = pf_dv, dF0 = pf_dF0;
                    const int pv = pf_pv;
                    const float du = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), 8));
                    const float nd = du + wl;
                    const bool better = nd < dv;
                    const uint32_t imp = (uint32_t)__builtin_amdgcn_ballot_w64(better);
                    const uint32_t push = imp & (uint32_t)__builtin_amdgcn_ballot_w64(pv < 16);
                    const int pu = __builtin_amdgcn_readlane(pv, 8) & 0xf;  // u leaves the queue (pyx:92)
                    const int th = __builtin_amdgcn_readfirstlane(pf_third);
                    const uint32_t odd = ((uint32_t)__builtin_amdgcn_ballot_w64(v == F0) & imp) |
                                         ((uint32_t)__builtin_amdgcn_ballot_w64(nd < dF0) & push);
                    if (count >= 3 && odd == 0u) {
                        Li[u] = (uint8_t)pu;
                        if (better) { Ld[v] = nd; Li[v] = pbits; }
                        if (push) {
                            const int rank = (int)__builtin_amdgcn_mbcnt_lo(push, 0u);
                            int slot = qt + rank;
                            slot = slot >= ring ? slot - ring : slot;
                            if ((push >> lane) & 1u) Lq[slot] = (uint16_t)v;
                            qt += __builtin_popcount(push);
                            qt = qt >= ring ? qt - ring : qt;
                            count += __builtin_popcount(push);
                        }
                        front = F0;
                        second = th;
                        pf_issue(F0, th, q2 + 1 == ring ? 0 : q2 + 1);
                    } else {
                        Li[u] = (uint8_t)pu;
                        int nf = F0, nsecond = th;
                        if (imp) {
                            if (better) { Ld[v] = nd; Li[v] = pbits; }
                            if (push) {
                                // F0 (queued, so never pushed) lowered by edge k: later pushes compare with its
                                // new distance while it is still the front.  With an empty queue F0 is stale.
                                const uint32_t fm = count > 0 ? (uint32_t)__builtin_amdgcn_ballot_w64(v == F0) & imp : 0u;
                                uint32_t todo = push | fm;
                                int fr = count > 0 ? F0 : -1;  // the front after the pop (-1: the queue is empty)
                                uint32_t dfr = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(dF0));
                                do {
                                    const int k = __builtin_ctz(todo);
                                    todo &= todo - 1;
                                    const int vk = __builtin_amdgcn_readlane(v, k);
                                    const uint32_t ndk = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(nd), k);
                                    if ((fm >> k) & 1u) {
                                        if (fr == F0) dfr = ndk;
                                        continue;
                                    }
                                    int content = vk;
                                    if (fr < 0) {  // the first push into an empty queue is the front (qh == qt)
                                        fr = vk;
                                        dfr = ndk;
                                    } else if (ndk < dfr) {  // SLF: swap with the front (pyx:104-107)
                                        content = fr;
                                        Lq[qh] = (uint16_t)vk;
                                        fr = vk;
                                        dfr = ndk;
                                    }
                                    Lq[qt] = (uint16_t)content;
                                    nsecond = qt == q2 ? content : nsecond;  // the slot after the front was empty
                                    qt = qt + 1 == ring ? 0 : qt + 1;
                                    count++;
                                } while (todo);
                                nf = fr;
                            }
                        }
                        front = nf;
                        second = nsecond;
                        pf_issue(nf, nsecond, q2 + 1 == ring ? 0 : q2 + 1);
                    }
                    --left;
                    if constexpr (SIMAPS_SPFA_RING > 0)
                        if (count > ring && lane == 0) fault_or(sh.fault, SIMAPS_FAULT_ROUNDS);  // (diagnostic ring overflowed)
                    if (min(count, left) <= 0) break;
                    continue;
                    }
#endif
                    // (front / second are wave-uniform: keep them in SGPRs across the loop)
                    const int u = __builtin_amdgcn_readfirstlane(front);
                    qh = qn;
                    count--;                           // entries queue[qh .. qt) after the pop
                    const int F0 = __builtin_amdgcn_readfirstlane(second);  // the next front (valid if count >= 1)
                    const int q2 = qh + 1 == ring ? 0 : qh + 1;
                    qn = q2;
                    const int v = u + doff;
                    // one round of reads (in-order LDS sees this wave's earlier writes); the ballots below
                    // consume them together.  Lane 8's v is u: its pin read is u's (parent bits to keep)
                    // and its distance read is u's (no separate read of dist[u]).
                    const float dv = Ld[v];
                    const float du = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), 8));
                    const int pv = Li[v];
                    // the front's distance before this pop's relaxations (F0 is a ring slot's content, a cell
                    // index, always: unused when count == 0)
                    const float dF0 = Ld[F0];
                    const int third = Lq[q2];          // queue[qh + 1]: the next pop's second (if count >= 2)
                    const float nd = du + wl;
                    // (lanes >= 8: v = u, so nd = du + 1 > dv: never `better`; no lane test needed)
                    const bool better = nd < dv;
                    const uint64_t imp = __builtin_amdgcn_ballot_w64(better);
                    // not queued: bit 4 clear, i.e. pv < 16 (a pin byte is at most 0x18: one compare)
                    const uint64_t notq = __builtin_amdgcn_ballot_w64(pv < 16);
                    Li[u] = (uint8_t)(__builtin_amdgcn_readlane(pv, 8) & 0xf);  // u leaves the queue (pyx:92)
                    int nf = F0, nsecond = __builtin_amdgcn_readfirstlane(third);
                    if (imp) {
                        if (better) { Ld[v] = nd; Li[v] = pbits; }
                        const uint64_t push = imp & notq;
                        if (push) {
                            // The pushes of this pop, in edge order (pyx:104-111): each goes to the tail and
                            // swaps with the front if its distance is below the front's at that moment.  The
                            // front's distance seen by edge k is F0's, lowered by this pop only if F0 is the
                            // head of an earlier edge jf < k (F0 is queued, so never pushed, but it may be
                            // relaxed) -- until the first push that beats it (js); from then on it is the
                            // running minimum of the pushed distances from js on.  A swapping push's slot
                            // receives the previous front (F0 or the previous swapping push's vertex); the last
                            // swapper ends at the front.
                            const int np = __popcll(push);
                            // F0 as the head of an edge this pop IMPROVED (lane jf): only then does its
                            // distance change for the later edges.  (Lanes >= 8 have v = u != F0 and never
                            // improve; with an empty queue F0 is stale, but that case ignores jf.)
                            const uint64_t fmi = __builtin_amdgcn_ballot_w64(v == F0) & imp;
                            const int jf = fmi ? __builtin_ctzll(fmi) : 64;
                            const float dafter = fmi ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nd), jf)) : dF0;
                            if (np == 1 && count > 0) {
                                // one push (the common case): a scalar decision, no scans
                                const int p1 = __builtin_ctzll(push);
                                const int vp = __builtin_amdgcn_readlane(v, p1);
                                const float ndp = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nd), p1));
                                const bool sw = ndp < (p1 > jf ? dafter : dF0);
                                const int content = sw ? F0 : vp;
                                Lq[qt] = (uint16_t)content;
                                if (sw) { Lq[qh] = (uint16_t)vp; nf = vp; }
                                if (count == 1) nsecond = content;  // the tail slot was queue[qh + 1]
                                qt = qt + 1 == ring ? 0 : qt + 1;
                                count++;
                            } else {
                                const bool isP = (push >> lane) & 1;
                                const int rank = __popcll(push & ((1ull << lane) - 1));
                                uint64_t cand = push;
                                int Fq = F0;
                                float dbefore = dF0, dseen = dafter;
                                if (count == 0) {  // the queue was empty: the first push becomes the front
                                    const int p1 = __builtin_ctzll(push);
                                    Fq = __builtin_amdgcn_readlane(v, p1);
                                    dbefore = dseen = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nd), p1));
                                    cand &= cand - 1;
                                }
                                const bool isC = (cand >> lane) & 1;
                                const uint64_t sF0 = __ballot(isC && nd < (lane > jf ? dseen : dbefore));
                                int content = v, newfront = Fq;
                                if (sF0) {
                                    const int js = __builtin_ctzll(sF0);
                                    // exclusive prefix minimum of nd over the candidate lanes in [js, lane) (DPP
                                    // row shifts: lanes 0-7 lie in one row)
                                    float y = (isC && lane >= js) ? nd : INFINITY;
        #define SPFA_SHR(x, n, old) __builtin_amdgcn_update_dpp((old), (x), 0x110 + (n), 0xf, 0xf, false)
        #define SPFA_SHRF(x, n) __int_as_float(SPFA_SHR(__float_as_int(x), n, (int)INF_BITS))
                                    y = fminf(y, SPFA_SHRF(y, 1));
                                    y = fminf(y, SPFA_SHRF(y, 2));
                                    y = fminf(y, SPFA_SHRF(y, 4));
                                    const float pm = SPFA_SHRF(y, 1);
                                    const bool sw = isC && (lane == js || (lane > js && nd < pm));
                                    const uint64_t swm = __ballot(sw);
                                    // the previous swapper's vertex: exclusive "last valid" scan of v over swappers
                                    int z = sw ? v : -1, zs;
                                    zs = SPFA_SHR(z, 1, -1); z = z >= 0 ? z : zs;
                                    zs = SPFA_SHR(z, 2, -1); z = z >= 0 ? z : zs;
                                    zs = SPFA_SHR(z, 4, -1); z = z >= 0 ? z : zs;
                                    const int prev = SPFA_SHR(z, 1, -1);
        #undef SPFA_SHRF
        #undef SPFA_SHR
                                    if (sw) content = prev >= 0 ? prev : Fq;
                                    newfront = __builtin_amdgcn_readlane(v, 63 - __builtin_clzll(swm));
                                }
                                const int slot = qt + rank < ring ? qt + rank : qt + rank - ring;
                                if (isP) Lq[slot] = (uint16_t)content;
                                if (sF0) Lq[qh] = (uint16_t)newfront;  // after the lanes' stores (in the empty case qh is p1's slot)
                                if (count <= 1) {  // the pushes wrote queue[qh + 1]: the next pop's second
                                    const uint64_t at = __ballot(isP && slot == q2);
                                    if (at) nsecond = __builtin_amdgcn_readlane(content, __builtin_ctzll(at));
                                }
                                qt = qt + np < ring ? qt + np : qt + np - ring;
                                count += np;
                                nf = newfront;
                            }
                        }
                    }
                    front = nf;
                    second = nsecond;
                    --left;
                    if constexpr (SIMAPS_SPFA_RING > 0)
                        if (count > ring && lane == 0) fault_or(sh.fault, SIMAPS_FAULT_ROUNDS);  // (diagnostic ring overflowed)
                    if (min(count, left) <= 0) break;  // (count, left >= 0)
                }
                pops = lim - left;
                if (count <= 0 || pops >= SIMAPS_POP_CAP) break;
                // (EARLY only: lim < SIMAPS_POP_CAP) early exit: every 32 pops, is the target at its final
                // distance and then every vertex of its parent chain?  The chain is walked in LDS (one
                // round per step), 64 vertices to a batch, each batch's distances compared with the
                // fixpoint in one lane-parallel global read.
                lim = pops + 32;
                if (OVL && !have_fin &&
                    __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sh.swept, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                    have_fin = true;
                    finT = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sh.finT)));
                    if (finT == INFINITY || finT == -INFINITY) { early = true; break; }
                }
                if (EARLY && have_fin && __builtin_amdgcn_readfirstlane(__float_as_int(Ld[tv])) == __float_as_int(finT)) {
                    tfinal = true;  // (from now on the asm loop leaves the target checks to this code)
                    int v = tv, pv = Li[tv], st = 0;
                    bool ok = true;
                    while (ok && v != su) {
                        int mine = -1;
                        for (int k = 0; k < 64 && v != su; k++, st++) {
                            const int pd = pv & 0xf;
                            if (!pd || st >= cells) { ok = false; break; }
                            v -= __builtin_amdgcn_readlane(doff, pd - 1);
                            if (lane == k) mine = v;
                            pv = Li[v];
                        }
                        if (ok && __ballot(mine >= 0 && Ld[mine] != (OVL ? fix[mine] : gfin[mine]))) ok = false;
                    }
                    // drain the walk's LDS reads here: left pending on any exit of this block, they make
                    // the compiler wait for every LDS access at the loop's back edge on the common
                    // (no-check) path too
                    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
                    if (ok) { early = true; break; }
                    lim = pops + gap;  // not yet: look again later, at doubling intervals (a failed walk
                    gap *= 2;          // costs ~a chain's length of LDS rounds)
                }
                lim = lim < SIMAPS_POP_CAP ? lim : SIMAPS_POP_CAP;
            }
        if (lane == 0) {
            STAMP_VAL(7, pops);  // (stamp build: tools/path_bench.py reports ns per pop)
            if (count > 0 && !early) fault_or(sh.fault, SIMAPS_FAULT_ROUNDS);  // the pop cap stopped a live queue
        }
    }
    lds_barrier();
    if (tid == 0) STAMP_NB(3);
    // (4) dense path: parents from the target back to the source (pyx:131-138), as rect cells
    if (tid == 0) {
        int cnt = 0, v = tv;
        auto pack = [&](int c) { const int rr = c / pw; return (uint16_t)(((rr - 1) << 8) | (c - rr * pw - 1)); };
        if (run_spfa) {
            dense[cnt++] = pack(v);
            while (v != su) {
                const int p = pin[v] & 0xf;
                if (!p) break;
                v -= dir_off(p - 1, pw);
                dense[cnt++] = pack(v);
            }
        }
        sh.nseg = cnt;
    }
    lds_barrier();
    const int nd = sh.nseg;
    if (tid == 0) STAMP_NB(4);
    // (5) approximate_polygon(dense, tolerance=1) (skimage 0.18.3 measure/_polygon.py), one wave, on
    // the global (row, col) indices like the reference (the fp64 distances are not translation-exact)
    for (int k = tid; k < nd; k += PNT) chain[k] = (k == 0 || k == nd - 1) ? 1 : 0;
    lds_barrier();
    const int gi0 = sh.i0, gj0 = sh.j0;
    if (tid < 64 && nd > 0) {
        int sp = 0, iters = 0;
        if (lane == 0) stack[0] = (uint32_t)(nd - 1) << 16;
        sp = 1;
        while (sp > 0 && ++iters <= 2 * nd) {  // each pop either splits at a new chain point or ends
            sp--;
            const uint32_t se = stack[sp];
            const int start = (int)(se & 0xffff), end = (int)(se >> 16);
            const int r0 = (dense[start] >> 8) + gi0, c0 = (dense[start] & 0xff) + gj0;
            const int r1 = (dense[end] >> 8) + gi0, c1 = (dense[end] & 0xff) + gj0;
            const long dr = r1 - r0, dc = c1 - c0;
            const double ang = -atan2((double)dr, (double)dc);
            const double sn = sin(ang), cs = cos(ang);
            const double sdist = (double)c0 * sn + (double)r0 * cs;
            double best = -1.0;
            int besti = -1;
            for (int k = start + 1 + lane; k < end; k += 64) {
                const int rr = (dense[k] >> 8) + gi0, cc = (dense[k] & 0xff) + gj0;
                const long dr0 = rr - r0, dc0 = cc - c0, dr1 = rr - r1, dc1 = cc - c1;
                const bool perp = dr0 * dr + dc0 * dc > 0 && -dr1 * dr - dc1 * dc > 0;
                double d;
                if (perp) d = fabs(((double)rr * cs + (double)cc * sn) - sdist);
                else d = fmin(sqrt((double)(dc0 * dc0 + dr0 * dr0)), sqrt((double)(dc1 * dc1 + dr1 * dr1)));
                if (d > best) { best = d; besti = k; }  // per lane: first maximum (ascending k)
            }
            // wave argmax with the first index on ties (np.argmax)
            for (int off = 32; off > 0; off >>= 1) {
                const double ob = __shfl_xor(best, off);
                const int oi = __shfl_xor(besti, off);
                if (ob > best || (ob == best && oi >= 0 && (besti < 0 || oi < besti))) { best = ob; besti = oi; }
            }
            if (best > 1.0) {  // np.any(segment_dists > tolerance)
                const int ne = besti;
                if (lane == 0) {
                    stack[sp] = (uint32_t)ne | ((uint32_t)end << 16);
                    stack[sp + 1] = (uint32_t)start | ((uint32_t)ne << 16);
                    chain[ne] = 1;
                }
                sp += 2;
            }
        }
    }
    lds_barrier();
    if (tid == 0) STAMP_NB(5);
    // (6) line-of-sight pruning on the grid (pyx:143-150), then reversed (pyx:152)
    if (tid < 64) {
        int m = 0;  // sparse points = chain-flagged dense points, in order
        for (int k0 = 0; k0 < nd; k0 += 64) {
            const int k = k0 + lane;
            const bool f = k < nd && chain[k];
            const uint64_t b = __ballot(f);
            if (f) sparse[m + __popcll(b & ((1ull << lane) - 1))] = dense[k];
            m += __popcll(b);
        }
        int cnt = 0;
        if (m > 0) {
            if (lane == 0) outp[0] = sparse[0];
            cnt = 1;
            for (int k = 1; k < m - 1; k++) {
                const int a = outp[cnt - 1], b2 = sparse[k + 1];
                if (!line_free(sh, S, (a >> 8) + gi0, (a & 0xff) + gj0, (b2 >> 8) + gi0, (b2 & 0xff) + gj0, line_mask)) {
                    if (lane == 0) outp[cnt] = sparse[k];
                    cnt++;
                }
            }
            if (m > 1) {
                if (lane == 0) outp[cnt] = sparse[m - 1];
                cnt++;
            }
        }
        if (lane == 0) STAMP_NB(6);
        return cnt;
    }
    return 0;
}

template <int CELLS, bool EARLY, bool OVL>
__global__ void __launch_bounds__(PNT) path_kernel(simaps_config cfg, Geometry geo, const simaps_agent *__restrict__ agents,
                                                   const simaps_env *__restrict__ envs,
                                                   const simaps_robot *__restrict__ robots,
                                                   const uint8_t *__restrict__ occupancy,
                                                   const double *__restrict__ sources, const double *__restrict__ targets,
                                                   int max_pts, double *__restrict__ out_xy, int *__restrict__ out_n,
                                                   float *scratch, unsigned *fault)
{
    __shared__ __attribute__((aligned(16))) char smem[path_lds_bytes<CELLS, OVL>()];
    PathHdr &sh = *reinterpret_cast<PathHdr *>(smem);
    SsspScratch &S = *reinterpret_cast<SsspScratch *>(smem + OFF_PS);
    const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int H = cfg.H, W = cfg.W;
    const Group g{tid, PNT, nullptr, PNT / 64};
    if (tid == 0) STAMP_NB(0);
    const simaps_agent ag = agents[n];
    const double sx = sources[2 * n], sy = sources[2 * n + 1], tx = targets[2 * n], ty = targets[2 * n + 1];
    if (tid == 0) {
        bool bad;
        const int type = agent_robot_type(ag, envs, robots, bad);
        sh.fault = bad ? SIMAPS_FAULT_DESCRIPTOR : 0u;
        sh.h = cfg.room_h;
        sh.w = cfg.room_w;
        sh.i0 = cfg.room_i0;
        sh.j0 = cfg.room_j0;
        sh.r = geo.cspace_r[type];
        pos_to_pix(sx, sy, H, W, sh.src_q[0][0], sh.src_q[0][1]);
        pos_to_pix(tx, ty, H, W, sh.src_q[1][0], sh.src_q[1][1]);
        sh.nsrc = 2;
    }
    lds_barrier();
    build_cspace<PNT>(S, nullptr, sh.h, sh.w, sh.r, g, nullptr, 0, nullptr, occupancy + (size_t)ag.map_slot * H * W, H,
                      W, sh.i0, sh.j0);
    double *o = out_xy + (size_t)n * max_pts * 2;
    // (1) straight line on cspace_thin between the unsnapped pixels (envs.py:2484-2486)
    if (tid < 64) {
        const bool straight = line_free(sh, S, sh.src_q[0][0], sh.src_q[0][1], sh.src_q[1][0], sh.src_q[1][1], LINE_THIN);
        if (lane == 0) sh.flag[0] = straight;
    }
    lds_barrier();
    if (sh.flag[0]) {
        if (tid == 0) {
            o[0] = sx; o[1] = sy; o[2] = tx; o[3] = ty; out_n[n] = 2;
            post_faults(fault, sh.fault);
        }
        return;
    }
    // (2) snap both ends (envs.py:2489-2490)
    if (tid == 0) STAMP_NB(1);
    snap_sources(sh, S, 2, g);
    const uint16_t *outp;
    const int cnt = path_core<CELLS, EARLY, OVL>(sh, S, smem + OFF_PA, H, W, sh.src_ok[0] && sh.src_ok[1], LINE_CSPACE,
                                                 EARLY && !OVL ? scratch + (size_t)n * CELLS : nullptr, outp);
    if (tid < 64) {
        // (7) positions (envs.py:2494-2503); path[0] / path[-1] replaced by the given positions
        if (cnt < 2) {
            if (lane == 0) { o[0] = sx; o[1] = sy; o[2] = tx; o[3] = ty; out_n[n] = 2; }
        } else if (cnt > max_pts) {
            if (lane == 0) out_n[n] = -cnt;  // caller's buffer too small
        } else {
            for (int k = lane; k < cnt; k += 64) {
                const int pv = outp[cnt - 1 - k], pi = (pv >> 8) + sh.i0, pj = (pv & 0xff) + sh.j0;
                double x = ((pj + 0.5) - (double)W / 2) / PPM, y = ((double)H / 2 - (pi + 0.5)) / PPM;
                if (k == 0) { x = sx; y = sy; }
                if (k == cnt - 1) { x = tx; y = ty; }
                o[2 * k] = x;
                o[2 * k + 1] = y;
            }
            if (lane == 0) out_n[n] = cnt;
        }
        if (lane == 0) post_faults(fault, sh.fault);
    }
}

// GridGraph(grid).shortest_path(source, target) (shortest_paths.pyx:121-154) on raw grid cells, one
// workgroup per (grid, source, target): the same exact SPFA / parent walk / approximate_polygon as
// path_kernel, without the cspace, snap and straight-line steps of OccupancyMap.shortest_path, the
// line-of-sight pruning on the grid itself, and the waypoints returned as cells (target last).
template <int CELLS, bool EARLY, bool OVL>
__global__ void __launch_bounds__(PNT) grid_path_kernel(int H, int W, const uint8_t *__restrict__ grids,
                                                        const int32_t *__restrict__ sources,
                                                        const int32_t *__restrict__ targets, int wi0, int wj0, int wh,
                                                        int ww, int max_pts, int32_t *__restrict__ out_ij,
                                                        int32_t *__restrict__ out_n, float *scratch, unsigned *fault)
{
    __shared__ __attribute__((aligned(16))) char smem[path_lds_bytes<CELLS, OVL>()];
    PathHdr &sh = *reinterpret_cast<PathHdr *>(smem);
    SsspScratch &S = *reinterpret_cast<SsspScratch *>(smem + OFF_PS);
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint8_t *grid = grids + (size_t)b * H * W;
    const int si = sources[2 * b], sj = sources[2 * b + 1], ti = targets[2 * b], tj = targets[2 * b + 1];
    if (tid == 0) {
        sh.h = wh; sh.w = ww; sh.i0 = wi0; sh.j0 = wj0;
        sh.fault = 0u;
        const bool s_in = si >= wi0 && si < wi0 + wh && sj >= wj0 && sj < wj0 + ww;
        const bool t_in = ti >= wi0 && ti < wi0 + wh && tj >= wj0 && tj < wj0 + ww;
        // a source outside the window or blocked has no edges (pyx:56), and a target outside the
        // window is never reached: the parent walk stops at once and the path is [target]
        sh.flag[0] = s_in && t_in && grid[(size_t)si * W + sj] != 0;
        sh.src_s[0][0] = si; sh.src_s[0][1] = sj; sh.src_s[1][0] = ti; sh.src_s[1][1] = tj;
    }
    // free bits (grid != 0: the SPFA's vertices, pyx:47-56) and grid == 1 bits (line of sight)
    const int nwords = (ww + 63) >> 6;
    for (int item = wave; item < wh * 2; item += PNT / 64) {
        const int rr = item >> 1, wd = item & 1, c = wd * 64 + lane;
        const uint8_t v = (wd < nwords && c < ww) ? grid[(size_t)(wi0 + rr) * W + wj0 + c] : (uint8_t)0;
        const uint64_t mf = __ballot(v != 0), m1 = __ballot(v == 1);
        if (lane == 0) {
            if (wd == 0) { S.freeb[rr].lo = mf; S.dtab[0][rr].lo = m1; }
            else { S.freeb[rr].hi = mf; S.dtab[0][rr].hi = m1; }
        }
    }
    lds_barrier();
    int32_t *o = out_ij + (size_t)b * max_pts * 2;
    if (!sh.flag[0]) {
        if (tid == 0) { o[0] = ti; o[1] = tj; out_n[b] = 1; }
        return;
    }
    const uint16_t *outp;
    const int cnt = path_core<CELLS, EARLY, OVL>(sh, S, smem + OFF_PA, H, W, true, LINE_GRID_ONE,
                                                 EARLY && !OVL ? scratch + (size_t)b * CELLS : nullptr, outp);
    if (tid < 64) {
        if (cnt > max_pts) {
            if (lane == 0) out_n[b] = -cnt;  // caller's buffer too small
        } else {
            for (int k = lane; k < cnt; k += 64) {  // reversed (pyx:152): source first
                const int pv = outp[cnt - 1 - k];
                o[2 * k] = (pv >> 8) + wi0;
                o[2 * k + 1] = (pv & 0xff) + wj0;
            }
            if (lane == 0) out_n[b] = cnt;
        }
        if (lane == 0) post_faults(fault, sh.fault);
    }
}

// ------------------------------------------------------------------------------------------------
// Observation ingest: Robot.update_map minus the simulator (envs.py:925, 2056-2066): the camera frame
// -> point cloud (Camera.capture_image, envs.py:1927-1955) -> overhead map (highest point per pixel:
// argsort by z + last write) and occupancy map (obstacle points, OccupancyMap.update 2447-2450).
// numpy float32 semantics op for op; np.dot / np.linalg.norm of float32 3-vectors = float32 products
// summed in double (OpenBLAS sdot), np.cross = (a1 b2 - a2 b1, ...).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float dot3f(const float *a, const float *b)
{
    return (float)((((double)(a[0] * b[0])) + (double)(a[1] * b[1])) + (double)(a[2] * b[2]));
}

// Two passes, no recomputation and no reset pass:
//   ingest_points_kernel  grid (chunks of INGEST_PTS camera pixels, frames): each point once -- its
//                         map pixel, its obstacle bit (occupancy byte store) and its key
//                         (launch epoch 8 bits | monotone z bits 32 | camera pixel + 1 20 | seg code
//                         4).  The keys are max-reduced per map pixel in LDS over the chunk's
//                         bounding box of map pixels (direct-mapped, no hashing), then ONE global
//                         64-bit atomicMax per touched pixel of the box.  A chunk's 2048 points hit
//                         only 14-1021 distinct pixels (the near rows of a forward camera ~30), so
//                         atomics straight from the points serialised on a few L2 lines (547 us per
//                         256 frames); an LDS hash table cost 22 us of init / scan on top of the
//                         reduction (95 us).  A box larger than the LDS window uses a direct-mapped
//                         (cell tag, key) table in the same LDS.  The seg value (a sum of 1/8
//                         multiples < 2, exact in f32) travels as seg * 8 in the key's low 4 bits, so
//                         the winner's value needs no second look-up.  Each chunk also stores its box
//                         (boxes[n][chunk]).
//   ingest_resolve_kernel 8 workgroups per frame: per map row, the columns the chunk boxes cover, of
//                         the slot's key map: a key of this launch's epoch writes overhead = code / 8.
//                         Keys of earlier launches carry smaller epochs, so every key of this launch
//                         beats them in the atomicMax and nothing is ever zeroed again (the caller
//                         clears the key map when the epoch wraps, include/simaps.h).
// HBM per frame: 8 B per camera pixel (depth + seg) + 8 B per swept key + the pixel writes.
// (measured alternatives, 256 frames: 128- / 64-thread chunks +4 / +21 us, an 8192-entry window
// +30 us (LDS occupancy), workgroups looping over several chunks of a frame with the next chunk's
// loads in flight +4..28 us: the per-chunk barrier chain wants many chunks in flight, not fewer)
constexpr int INGEST_WG = 256, INGEST_PPT = 8, INGEST_PTS = INGEST_WG * INGEST_PPT;
__host__ __device__ constexpr int ingest_chunks(int hc, int wc) { return (hc * wc + INGEST_PTS - 1) / INGEST_PTS; }
#ifndef SIMAPS_INGEST_WIN
#define SIMAPS_INGEST_WIN 2048
#endif
constexpr int INGEST_WIN = SIMAPS_INGEST_WIN;  // LDS window entries (u64 keys) over a chunk's map-pixel box
constexpr int INGEST_MAX_WC = 1024, INGEST_MAX_ROWS = 32;  // camera width; camera rows one chunk spans
// A chunk's pixels k0 .. k0 + INGEST_PTS - 1 reach camera row k0 / Wc + 1 + (INGEST_PTS - 2) / Wc at most
// (k0 % Wc = Wc - 1): its row table index must stay below INGEST_MAX_ROWS.  Smallest such width: 67.
constexpr bool ingest_width_ok(int wc) { return wc >= 1 && wc <= INGEST_MAX_WC && 1 + (INGEST_PTS - 2) / wc < INGEST_MAX_ROWS; }
constexpr int ingest_min_width(int wc = 1) { return ingest_width_ok(wc) ? wc : ingest_min_width(wc + 1); }
static_assert(ingest_min_width() == 67, "include/simaps.h documents the camera width range [67, 1024]");
#ifndef SIMAPS_INGEST_RES_G
#define SIMAPS_INGEST_RES_G 8
#endif
#ifndef SIMAPS_INGEST_RES_ROWS
#define SIMAPS_INGEST_RES_ROWS 2
#endif
// resolve: INGEST_RES_G workgroups per frame, INGEST_RES_ROWS rows in flight per wave
constexpr int INGEST_RES_WG = 256, INGEST_RES_G = SIMAPS_INGEST_RES_G, INGEST_RES_ROWS = SIMAPS_INGEST_RES_ROWS;

// Camera.capture_image's frame (envs.py:1932-1940) in float32: position, principal, up, right.
__device__ __forceinline__ void camera_frame(const double *P, float *F)
{
    float cp[3], pr[3], cu[3], up[3], rt[3];
    for (int c = 0; c < 3; c++) {
        cp[c] = (float)P[c];
        pr[c] = (float)P[3 + c] - cp[c];
        cu[c] = (float)P[6 + c];
    }
    const float n1 = sqrtf(dot3f(pr, pr));
    for (int c = 0; c < 3; c++) pr[c] = pr[c] / n1;
    const float d = dot3f(cu, pr);
    for (int c = 0; c < 3; c++) up[c] = cu[c] - d * pr[c];
    const float n2 = sqrtf(dot3f(up, up));
    for (int c = 0; c < 3; c++) up[c] = up[c] / n2;
    rt[0] = pr[1] * up[2] - pr[2] * up[1];
    rt[1] = pr[2] * up[0] - pr[0] * up[2];
    rt[2] = pr[0] * up[1] - pr[1] * up[0];
    const float n3 = sqrtf(dot3f(rt, rt));
    for (int c = 0; c < 3; c++) {
        F[c] = cp[c];
        F[3 + c] = pr[c];
        F[6 + c] = up[c];
        F[9 + c] = rt[c] / n3;
    }
}

__device__ __forceinline__ int wave_min(int v)
{
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v)
{
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// Loads of a chunk: each lane owns INGEST_PPT consecutive camera pixels (one camera row segment;
// neighbouring pixels of the near rows land on one map pixel, so the lane max-merges runs first).
__device__ __forceinline__ void ingest_load(const float *db, const int32_t *raw, int k0, int NP, float (&dv)[INGEST_PPT],
                                            int (&rv)[INGEST_PPT])
{
    static_assert(INGEST_PPT % 4 == 0, "16-B loads per lane and array");
    if ((NP & 3) == 0 && k0 + INGEST_PPT <= NP) {  // 16-B aligned: frames start at n * NP, k0 % 4 == 0
        const float4 *d4 = reinterpret_cast<const float4 *>(db + k0);
        const int4 *r4 = reinterpret_cast<const int4 *>(raw + k0);
#pragma unroll
        for (int v = 0; v < INGEST_PPT / 4; v++) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            typedef int i4 __attribute__((ext_vector_type(4)));
            const f4 d = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(d4 + v));
            const i4 r = __builtin_nontemporal_load(reinterpret_cast<const i4 *>(r4 + v));
            dv[4 * v] = d.x, dv[4 * v + 1] = d.y, dv[4 * v + 2] = d.z, dv[4 * v + 3] = d.w;
            rv[4 * v] = r.x, rv[4 * v + 1] = r.y, rv[4 * v + 2] = r.z, rv[4 * v + 3] = r.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < INGEST_PPT; q++) {
            dv[q] = k0 + q < NP ? db[k0 + q] : 0.0f;
            rv[q] = k0 + q < NP ? raw[k0 + q] : 0;
        }
    }
}

// min (is_min) or max over the wave by DPP (quad, half-row and row mirrors, then the row
// broadcasts); lanes of rows a broadcast leaves out keep their value (op(v, v) = v)
template <class Op>
__device__ __forceinline__ int wave_reduce_dpp(int v, Op op)
{
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0xb1, 0xf, 0xf, false));   // quad_perm [1, 0, 3, 2]
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x4e, 0xf, 0xf, false));   // quad_perm [2, 3, 0, 1]
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xf, 0xf, false));  // row_half_mirror
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xf, 0xf, false));  // row_mirror: the row's result
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xa, 0xf, false));  // row_bcast15 -> rows 1, 3
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xc, 0xf, false));  // row_bcast31 -> rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_reduce_dpp(int v, bool is_min)
{
    return is_min ? wave_reduce_dpp(v, [](int a, int b) { return min(a, b); })
                  : wave_reduce_dpp(v, [](int a, int b) { return max(a, b); });
}
// two u16 halves at once (v_pk_min_u16 / v_pk_max_u16)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int pk_min_u16(int a, int b)
{
    return __builtin_bit_cast(int, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ int pk_max_u16(int a, int b)
{
    return __builtin_bit_cast(int, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}

// np.floor(v).astype(np.int32) then np.clip(., 0, n - 1) (envs.py:2440-2442) of an already floored
// float32 f: the hardware convert saturates and takes NaN to 0, med3 clamps, and a value >= 2^31
// (INT32_MIN in numpy, x86 cvttss2si) clips to 0
__device__ __forceinline__ int ingest_clip(float f, int n)
{
    int c;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(c) : "v"(f));
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(c) : "v"(c), "s"(n - 1));
    return f >= 2147483648.0f ? 0 : c;
}

// grid (chunks, frames); WCS: the column tables' stride (>= the camera width; 320 holds both reference
// cameras, 156 and 277 columns, in 4 KB: LDS decides how many chunks a CU holds)
template <int WCS>
__global__ void __launch_bounds__(INGEST_WG) ingest_points_kernel(
    simaps_config cfg, simaps_camera cam, const simaps_agent *__restrict__ agents,
    const simaps_seg_ids *__restrict__ seg_ids, const double *__restrict__ cam_params,
    const float *__restrict__ depth, const int32_t *__restrict__ seg_raw, uint8_t *__restrict__ occupancy,
    unsigned long long *__restrict__ keys, unsigned *__restrict__ boxes, unsigned epoch)
{
    __shared__ unsigned long long win[INGEST_WIN];
    // per chunk: A[c][j] = right[c] * pixel_x(j) + principal[c] (column j), Bt[c][i] = up[c] * pixel_y(i)
    // (row row0 + i): a point's ray t[c] = A[c][j] + Bt[c][i], the same float32 operations in the same
    // order as per point (capture_image, envs.py:1946-1950)
    // (A holds INGEST_PPT wrapped columns past Wc: A[c][Wc + t] = A[c][t], so a lane's 8 columns are
    // consecutive table entries even where its pixels wrap to the next row; segT: seg * 8 of body
    // ids -1 .. 254 at segT[id + 1])
    __shared__ float A[3][WCS + INGEST_PPT], Bt[3][INGEST_MAX_ROWS], Fs[3];
    __shared__ uint8_t segT[256];
    __shared__ int box[4];  // min i, -max i, min j, -max j of the chunk's map pixels
    const int n = blockIdx.y, tid = threadIdx.x;
    const int H = cfg.H, W = cfg.W, Hc = cam.height_px, Wc = cam.width_px, NP = Hc * Wc;
    const float *db = depth + (size_t)n * NP;
    const int32_t *raw = seg_raw + (size_t)n * NP;
    const int k0 = blockIdx.x * INGEST_PTS + tid * INGEST_PPT;
    float dv[INGEST_PPT];
    int rv[INGEST_PPT];
    // issue the chunk's loads first: the per-chunk tables below hide their latency
    ingest_load(db, raw, k0, NP, dv, rv);
    const simaps_agent ag = agents[n];
    const simaps_seg_ids ids = seg_ids[ag.env];
    const float c1 = (float)(cam.far_m * cam.near_m), cfar = (float)cam.far_m, cfn = (float)(cam.far_m - cam.near_m);
    const float cx2 = (float)cam.cx2, cy2 = (float)cam.cy2;
    // seg * 8 per body id (the reference's float sum of 1/8 multiples < 2 is exact: its integer sum)
    auto seg8_of = [&](int r) {
        int v = r == 0 ? 1 : 0;
        v += (r >= ids.min_obstacle && r <= ids.max_obstacle) ? 2 : 0;
        v += (ids.has_receptacle && r == ids.receptacle) ? 3 : 0;
        v += (r >= ids.min_cube && r <= ids.max_cube) ? 4 : 0;
        return v;
    };
    // per chunk once, by wave 0 alone (the pass is VALU-issue bound: the other waves' issue slots
    // go to other chunks): the camera frame and the column and row tables (envs.py:1932-1947; the
    // float32 divisions and products every point of a column / row would repeat)
    const int row0 = (blockIdx.x * INGEST_PTS) / Wc;
    if (tid < 64) {
        float F[12];
        camera_frame(cam_params + 9 * (size_t)n, F);
#pragma unroll
        for (int c = 0; c < 12; c++) F[c] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(F[c])));
        for (int j = tid; j < Wc + INGEST_PPT; j += 64) {
            const int jj = j < Wc ? j : j - Wc;
            const float px = cx2 * ((float)jj / (float)Wc - 0.5f);
#pragma unroll
            for (int c = 0; c < 3; c++) A[c][j] = F[3 + c] + px * F[9 + c];
        }
#pragma unroll
        for (int e = tid; e < 256; e += 64) segT[e] = (uint8_t)seg8_of(e - 1);
        if (tid < INGEST_MAX_ROWS) {
            const float py = cy2 * (0.5f - ((float)(row0 + tid) + 1.0f) / (float)Hc);
#pragma unroll
            for (int c = 0; c < 3; c++) Bt[c][tid] = py * F[6 + c];
        }
        if (tid < 3) Fs[tid] = F[tid];
        if (tid < 4) box[tid] = INT32_MAX;
    }
    const float h2 = (float)((double)H / 2), w2 = (float)((double)W / 2);
    const size_t base = (size_t)ag.map_slot * H * W;
    uint8_t *const occ = occupancy + base;
    {
        __syncthreads();
        float F[3];
#pragma unroll
        for (int c = 0; c < 3; c++) F[c] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(Fs[c])));
        // Per point, branch-free: cell[q] = map row << 16 | map column, or -1 (no point); key[q] as
        // below.  A lane whose 8 pixels all lie in the frame (every lane but the frame's last few)
        // takes the TAIL = false instance: no validity selects.  (A point past the end computes on
        // zero inputs and is dropped.)  No per-point branch, so the unrolled arrays are never copied
        // at branch joins.
        int cell[INGEST_PPT];
        unsigned long long key[INGEST_PPT];
        int cmin = -1, cmax = 0;  // the lane's (row, column) box, packed like cell: u16 halves
        // body ids all in the seg table's range -1 .. 254 (wave-uniform): a table look-up per point
        unsigned idor = 0;
#pragma unroll
        for (int q = 0; q < INGEST_PPT; q++) idor |= (unsigned)(rv[q] + 1);
        const bool ids_ok = __builtin_amdgcn_ballot_w64(idor >= 256u) == 0;
        auto points = [&](auto tail) {
            constexpr bool TAIL = decltype(tail)::value;
            const int i0 = k0 / Wc, j0 = k0 - i0 * Wc, ir0 = i0 - row0;  // (rows past the frame stay inside the table)
            // a full lane's 8 columns are the consecutive table entries j0 .. j0 + 7 (wrapped copies
            // past Wc); its points from q = Wc - j0 on lie in the next row
            float B0[3], B1[3];
#pragma unroll
            for (int c = 0; c < 3; c++) B0[c] = Bt[c][ir0], B1[c] = Bt[c][min(ir0 + 1, INGEST_MAX_ROWS - 1)];  // (B1 only matters below the last row)
            int i = i0, j = j0;
#pragma unroll
            for (int q = 0; q < INGEST_PPT; q++, j = (j + 1 == Wc) ? (i++, 0) : j + 1) {
                const int k = k0 + q;
                const bool valid = !TAIL || k < NP;
                const float dep = c1 / (cfar - cfn * dv[q]);
                float p[3];
                if constexpr (TAIL) {
#pragma unroll
                    for (int c = 0; c < 3; c++) p[c] = F[c] + dep * (A[c][j] + Bt[c][i - row0]);
                } else {
                    const bool nxt = q >= Wc - j0;
#pragma unroll
                    for (int c = 0; c < 3; c++) p[c] = F[c] + dep * (A[c][j0 + q] + (nxt ? B1[c] : B0[c]));
                }
                int s8;
                if (ids_ok) s8 = segT[rv[q] + 1];
                else s8 = seg8_of(rv[q]);
                int pi = ingest_clip(floorf(h2 - p[1] * 96.0f), H), pj = ingest_clip(floorf(w2 + p[0] * 96.0f), W);
                const int cq = (pi << 16) | pj;
                cell[q] = valid ? cq : -1;
                cmin = valid ? pk_min_u16(cmin, cq) : cmin, cmax = valid ? pk_max_u16(cmax, cq) : cmax;
                if (valid && s8 == 2) occ[(unsigned)__umul24(pi, W) + pj] = 1;  // np.isclose(seg, obstacle) (exact values)
                // np.argsort order by z: float bits made unsigned-monotone, NaN last; equal z -> later pixel
                const unsigned zb = __float_as_uint(p[2]);
                const unsigned zk = p[2] != p[2] ? 0xffffffffu : ((zb & 0x80000000u) ? ~zb : (zb | 0x80000000u));
                key[q] = ((unsigned long long)epoch << 56) | ((unsigned long long)zk << 24) | (((unsigned)(k + 1) << 4) | (unsigned)s8);
            }
            // runs of one map pixel inside the lane: the run's last entry carries the run's max key
#pragma unroll
            for (int q = 1; q < INGEST_PPT; q++) {
                const bool run = cell[q] == cell[q - 1] && (!TAIL || cell[q] >= 0);
                key[q] = run && key[q - 1] > key[q] ? key[q - 1] : key[q];
                cell[q - 1] = run ? -1 : cell[q - 1];
            }
        };
        if (k0 + INGEST_PPT <= NP) points(std::false_type{});
        else points(std::true_type{});
        // the chunk's box of map pixels
        cmin = wave_reduce_dpp(cmin, pk_min_u16), cmax = wave_reduce_dpp(cmax, pk_max_u16);
        const int imin = (unsigned)cmin >> 16, jmin = cmin & 0xffff, imax = (unsigned)cmax >> 16, jmax = cmax & 0xffff;
        if ((tid & 63) == 0 && imin <= imax)  // (a wave without points keeps cmin = 0xffff'ffff, cmax = 0)
            atomicMin(&box[0], imin), atomicMin(&box[1], -imax), atomicMin(&box[2], jmin), atomicMin(&box[3], -jmax);
        __syncthreads();
        const int bi = box[0], bj = box[2], bh = -box[1] - bi + 1, bw = -box[3] - bj + 1;
        const int area = bh * bw;  // block-uniform (a chunk holds >= 1 point)
        if (tid == 0)  // the chunk's box of map pixels [i0, i1) x [j0, j1), for the resolve sweep
            reinterpret_cast<uint4 *>(boxes)[(size_t)n * gridDim.x + blockIdx.x] =
                make_uint4((unsigned)bi, (unsigned)(bi + bh), (unsigned)bj, (unsigned)(bj + bw));
        if (area > INGEST_WIN) {
            // box past the window (a forward camera's far rows: ~2-3 points per pixel, spread wide;
            // global atomics per run instead measured 3 us more per 256 frames):
            // a direct-mapped table of HS (cell tag, key) slots in the window's LDS.
            // Each cell's tag is written by its points (any one wins); points whose cell owns the
            // slot max-reduce there, the others (collisions) go straight to the global key map;
            // then one global atomic per used slot.
            constexpr int HS = INGEST_WIN * 2 / 3;  // keys (8 B) + tags (4 B) in the window's LDS
            unsigned long long *hk = win;
            int *ht = reinterpret_cast<int *>(win + HS);
            // slot: the cell's index in the box (row-major) mod HS -- neighbouring cells of a row
            // take neighbouring slots (the packed cell itself mod HS would fold rows 16 columns apart
            // onto one slot)
            auto slot = [&](int c) { return (unsigned)(((c >> 16) - bi) * bw + ((c & 0xffff) - bj)) % HS; };
            for (int e = tid; e < HS; e += INGEST_WG) hk[e] = 0ull, ht[e] = -1;
            __syncthreads();
#pragma unroll
            for (int q = 0; q < INGEST_PPT; q++)
                if (cell[q] >= 0) ht[slot(cell[q])] = cell[q];
            __syncthreads();
#pragma unroll
            for (int q = 0; q < INGEST_PPT; q++)
                if (cell[q] >= 0) {
                    const int h = slot(cell[q]);
                    if (ht[h] == cell[q]) atomicMax(&hk[h], key[q]);
                    else atomicMax(&keys[base + (cell[q] >> 16) * W + (cell[q] & 0xffff)], key[q]);
                }
            __syncthreads();
            for (int e = tid; e < HS; e += INGEST_WG) {
                const unsigned long long v = hk[e];
                if (v) atomicMax(&keys[base + (ht[e] >> 16) * W + (ht[e] & 0xffff)], v);
            }
            return;
        }
        for (int e = tid; e < area; e += INGEST_WG) win[e] = 0ull;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < INGEST_PPT; q++)
            if (cell[q] >= 0) atomicMax(&win[((cell[q] >> 16) - bi) * bw + ((cell[q] & 0xffff) - bj)], key[q]);
        __syncthreads();
        // the window's entries e = tid + m * INGEST_WG as (row, column) of the box, stepped without
        // a division per entry
        const int qs = INGEST_WG / bw, rs = INGEST_WG - qs * bw;
        int di = tid / bw, dj = tid - di * bw;
        for (int e = tid; e < area; e += INGEST_WG) {
            const unsigned long long v = win[e];
            if (v) atomicMax(&keys[base + (size_t)((bi + di) * W + bj + dj)], v);
            di += qs, dj += rs;
            if (dj >= bw) dj -= bw, di++;
        }
    }
}

// grid (INGEST_RES_G, frames): per map row of the frame, only the columns its chunk boxes cover --
// the union of the boxes that contain the row, one interval (a forward camera's boxes follow its
// viewing wedge: ~half of the frame's bounding box).  Rows are dealt round-robin over the frame's
// INGEST_RES_G * 4 waves, two rows in flight per wave; the lanes sweep a row's columns.  Each wave
// reads the chunk boxes itself (lane c: box c), so no barrier.
// ZERO (simaps_ingest's epoch 0, the graph-replayable mode): the launch's keys carry tag 1 on a key
// map that is all zero on entry, and every nonzero key read here is zeroed again, so the map is all
// zero on exit -- every replay of a captured launch starts from the same state.
template <bool ZERO>
__global__ void __launch_bounds__(INGEST_RES_WG) ingest_resolve_kernel(
    simaps_config cfg, const simaps_agent *__restrict__ agents, float *__restrict__ overhead,
    unsigned long long *__restrict__ keys, const unsigned *__restrict__ boxes, int nch, unsigned epoch)
{
    const int n = blockIdx.y, lane = threadIdx.x & 63, W = cfg.W;
    const int gw = blockIdx.x * (INGEST_RES_WG / 64) + (threadIdx.x >> 6), nw = INGEST_RES_G * (INGEST_RES_WG / 64);
    const uint4 *bx = reinterpret_cast<const uint4 *>(boxes) + (size_t)n * nch;
    // lane c < 64 holds box c (an empty box for c >= nch); more than 64 boxes (cameras over 131 k
    // pixels) are re-read per row below
    uint4 b0 = lane < nch ? bx[lane] : make_uint4(0x7fffffffu, 0u, 0x7fffffffu, 0u);
    const int fi0 = wave_reduce_dpp((int)b0.x, true), fi1 = wave_reduce_dpp((int)b0.y, false);
    int ri0 = fi0, ri1 = fi1;
    for (int c = 64 + lane; c < nch; c += 64) ri0 = min(ri0, (int)bx[c].x), ri1 = max(ri1, (int)bx[c].y);
    if (nch > 64) ri0 = wave_reduce_dpp(ri0, true), ri1 = wave_reduce_dpp(ri1, false);
    // the interval [lo, hi) of row r: the hull of the boxes containing r
    auto extent = [&](int r, int &lo, int &hi) {
        const bool in = (int)b0.x <= r && r < (int)b0.y;
        int a = in ? (int)b0.z : INT32_MAX, z = in ? (int)b0.w : 0;
        for (int c = 64 + lane; c < nch; c += 64) {
            const uint4 q = bx[c];
            if ((int)q.x <= r && r < (int)q.y) a = min(a, (int)q.z), z = max(z, (int)q.w);
        }
        lo = wave_reduce_dpp(a, true), hi = wave_reduce_dpp(z, false);
        if (hi <= lo) lo = hi = 0;  // no box holds the row
    };
    const size_t base = (size_t)agents[n].map_slot * cfg.H * W;
    constexpr int R = INGEST_RES_ROWS, U = 2;  // rows in flight; columns per lane and row in flight
    for (int r = ri0 + gw; r < ri1; r += R * nw) {
        int lo[R], hi[R], wmax = 0;
#pragma unroll
        for (int t = 0; t < R; t++) {
            lo[t] = hi[t] = 0;
            if (r + t * nw < ri1) extent(r + t * nw, lo[t], hi[t]);
            wmax = max(wmax, hi[t] - lo[t]);
        }
        for (int c0 = 0; c0 < wmax; c0 += 64 * U) {
            size_t idx[R * U];
            unsigned long long kv[R * U];
#pragma unroll
            for (int u = 0; u < R * U; u++) {
                const int t = u / U, c = lo[t] + c0 + (u % U) * 64 + lane;
                idx[u] = base + (size_t)(r + t * nw) * W + c;
                kv[u] = c < hi[t] ? keys[idx[u]] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < R * U; u++) {
                if ((unsigned)(kv[u] >> 56) == epoch) overhead[idx[u]] = (float)(kv[u] & 15ull) * 0.125f;
                if (ZERO && kv[u]) keys[idx[u]] = 0ull;
            }
        }
    }
}

#ifndef SIMAPS_DEVICE_ONLY
#include "grid_large.h"
#include "occupancy_map.h"
#include "global_maps.h"
#endif

}  // namespace

#ifndef SIMAPS_DEVICE_ONLY
// =================================================================================================
// C ABI
// =================================================================================================
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <mutex>
#include <vector>

namespace {
thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

// The process-wide device fault word (include/simaps.h SIMAPS_FAULT_*): SIMAPS_NFAULT flags in
// fine-grained (coherent) host memory that every device can write without a copy, read by the next
// compute call without synchronising.  Allocated on first use; never freed (process lifetime).
std::once_flag g_fault_once;
volatile unsigned *g_fault_host = nullptr;
unsigned *g_fault_dev = nullptr;

unsigned *fault_word()
{
    std::call_once(g_fault_once, [] {
        void *h = nullptr;
        if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
            return;
        memset(h, 0, 64);
        void *d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return;
        g_fault_host = static_cast<volatile unsigned *>(h);
        g_fault_dev = static_cast<unsigned *>(d);
    });
    return g_fault_dev;
}

unsigned read_faults(bool clear)
{
    unsigned f = 0;
    if (!g_fault_host) return 0;
    for (int k = 0; k < SIMAPS_NFAULT; k++) {
        // clear with an exchange: a fault posted by a launch still in flight between a read and a
        // separate store of 0 would be erased unreported
        const unsigned v = clear ? __atomic_exchange_n(&g_fault_host[k], 0u, __ATOMIC_ACQ_REL)
                                 : __atomic_load_n(&g_fault_host[k], __ATOMIC_ACQUIRE);
        if (v) f |= 1u << k;
    }
    return f;
}

// Entry check of every compute call: a fault posted by an earlier launch fails this call (once).
int pending_faults()
{
    if (!fault_word()) return fail(SIMAPS_EHIP, "could not allocate the host-mapped fault word");
    const unsigned f = read_faults(true);
    if (!f) return 0;
    return fail(SIMAPS_EDEVICE, "an earlier launch reported device fault bits 0x%x (%s%s%s): its outputs are invalid", f,
                f & SIMAPS_FAULT_TIMEOUT ? "barrier timeout " : "", f & SIMAPS_FAULT_ROUNDS ? "SSSP round cap " : "",
                f & SIMAPS_FAULT_DESCRIPTOR ? "descriptor clamped" : "");
}

// Robot geometry with the reference's own expressions (envs.py:802-810, 1060, 1280, 2218-2242, 2421).
Geometry make_geometry()
{
    Geometry g;
    const double HALF_WIDTH = 0.03, BACKPACK_OFFSET = -0.0135, BASE_LENGTH = 0.065, CUBE_WIDTH = 0.044;
    const double bl[4] = {BASE_LENGTH, BASE_LENGTH + 0.005, BASE_LENGTH + 0.006, BASE_LENGTH};
    for (int t = 0; t < 4; t++) {
        const double ee = BACKPACK_OFFSET + bl[t];
        const double radius = std::sqrt(HALF_WIDTH * HALF_WIDTH + ee * ee);
        g.base_length[t] = bl[t];
        g.cspace_r[t] = (int)std::floor(radius * 96.0);
        g.mask_width[t] = (int)std::ceil(2 * radius * 96.0);
        g.mask_start[t] = (int)std::floor(96 / 2.0 - g.mask_width[t] / 2.0);
    }
    g.cube_w = (int)std::ceil(CUBE_WIDTH * 96.0);
    g.pad = 0;
    g.half_width = HALF_WIDTH;
    g.half_width_sq = HALF_WIDTH * HALF_WIDTH;
    g.backpack_offset = BACKPACK_OFFSET;
    g.cube_half = CUBE_WIDTH / 2;
    g.cube_width = CUBE_WIDTH;
    g.cube_base = (BACKPACK_OFFSET + BASE_LENGTH) + (-0.007);  // LiftingRobot END_EFFECTOR + LIFTED_CUBE_OFFSET
    for (int m = 0; m < 5; m++) {
        const int t = m < 4 ? m : SIMAPS_LIFTING;
        const bool cube = m == 4;
        const int st = g.mask_start[t], wd = g.mask_width[t];
        g.mrow0[m] = cube ? st - g.cube_w : st;
        g.mcol0[m] = st;
        g.mnrows[m] = (st + wd) - g.mrow0[m];
        g.mncols[m] = wd;
        for (int r = 0; r < 24; r++) {
            uint32_t bits = 0;
            for (int c = 0; c < wd && r < g.mnrows[m]; c++)
                if (mask_bit(g, t, cube, g.mrow0[m] + r, g.mcol0[m] + c)) bits |= 1u << c;
            g.mbits[m][r] = bits;
        }
    }
    return g;
}

// The robot geometry never changes: computed once per process (the mask tables are ~2,000 fp64
// mask_bit evaluations, which every launch used to repeat on the host).
const Geometry &geometry()
{
    static const Geometry g = make_geometry();
    return g;
}

// Path kernel choice (simaps_path_mode).  1: compact.  2: early exit (the SSSP fixpoint first, then the
// SPFA only until the target's parent chain is final; same LDS footprint and pop loop as compact, so it
// pays its sweeps, ~15 us small rooms / ~26 us large, and chain checks: measured 0.7-1.05x the compact
// launch time for targets across the room and 0.5-0.95x for targets in the robot's local map, DESIGN.md
// section 5).  3: early exit with the sweeps overlapped (OVL: on waves 1-3 beside the SPFA, the
// fixpoint in LDS -- no pool scratch, so graph capture keeps it -- at 2 small-room / 1 large-room
// queries per CU instead of 4 / 2).  0, automatic: OVL while the launch is resident at once at OVL's
// residency (N <= CUs x per-CU), else 2 (compact when the launch is being captured).
std::atomic<int> g_path_mode{0};
enum PathKind { PK_COMPACT, PK_EARLY, PK_OVL };
int device_cus()
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}
PathKind path_kind(int n, bool small)
{
    switch (g_path_mode.load()) {
    case 1: return PK_COMPACT;
    case 2: return PK_EARLY;
    case 3: return PK_OVL;
    default: break;
    }
    const int per = small ? path_per_cu<PATH_SMALL_CELLS, true>() : path_per_cu<SIMAPS_MAX_ROOM_CELLS, true>();
    return (long)n <= (long)device_cus() * per ? PK_OVL : PK_EARLY;
}

// Device scratch of the early-exit path kernels (the SSSP fixpoint, CELLS f32 per query): stream-
// ordered, taken from a private memory pool of the device right before the launch
// (hipMallocFromPoolAsync on the launch stream) and handed back right after it (hipFreeAsync on the
// same stream), so no buffer is ever shared between launches, threads or streams, and nothing is
// synchronised.  The pool is this library's own (created once per device, release threshold 256 MiB so
// it keeps the path scratch: after the first launches this is a pool hit); the device's default pool,
// which other libraries in the process allocate from, is left as it was.  A launch being captured into
// a graph gets none and takes the compact kernels (same results) instead.
struct PathScratch {
    float *p = nullptr;
    hipStream_t st = nullptr;
    PathScratch() = default;
    PathScratch(const PathScratch &) = delete;
    PathScratch &operator=(const PathScratch &) = delete;
    ~PathScratch()
    {
        if (p) (void)hipFreeAsync(p, st);  // ordered after the launch that uses it
    }
};
std::once_flag g_pool_once[64];
hipMemPool_t g_pool[64] = {};
bool pool_alloc(PathScratch &ps, hipStream_t st, size_t bytes)
{
    int dev = 0;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || hipStreamIsCapturing(st, &cap) != hipSuccess ||
        cap != hipStreamCaptureStatusNone)
        return false;
    // An error left pending by the caller stays pending for the launch's own check: no scratch then
    // (the compact kernels run), and nothing here clears it.
    if (hipPeekAtLastError() != hipSuccess) return false;
    std::call_once(g_pool_once[dev], [dev] {
        hipMemPoolProps props = {};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
            (void)hipGetLastError();  // (only this call's error: none was pending above)
            return;
        }
        // Keep up to 256 MiB reserved across synchronisations: the early-exit scratch (CELLS f32
        // per query, 9 MB for 256 queries at the room limit) stays a pool hit, while the
        // large-window GridGraph scratch (~32 B per cell per query: GB on multi-Mcell grids) goes back
        // to the device at the next synchronisation instead of staying reserved for the process.
        uint64_t keep = 256ull << 20;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        g_pool[dev] = pool;
    });
    if (!g_pool[dev]) return false;
    void *p = nullptr;
    if (hipMallocFromPoolAsync(&p, bytes, g_pool[dev], st) != hipSuccess) {
        (void)hipGetLastError();  // (only this call's error)
        return false;
    }
    ps.p = (float *)p;
    ps.st = st;
    return true;
}
// the early-exit path kernels' scratch: none (the compact kernels run instead) when it cannot be had
void path_scratch(PathScratch &ps, hipStream_t st, size_t bytes) { (void)pool_alloc(ps, st, bytes); }

// the LDS-resident GridGraph kernels' window limit (include/simaps.h); beyond it grid_large.h
bool window_fits_lds(int wh, int ww)
{
    return ww <= SIMAPS_MAX_ROOM_W && wh <= MAX_ROWS && (wh + 2) * ((ww + 2) | 1) <= SIMAPS_MAX_ROOM_CELLS;
}

// the large-window fixpoint: the tiled kernel up to GT_MAXT tiles (windows up to ~3,968^2 cells), the
// whole-window sweeps beyond (SIMAPS_GL_TILE=0: always the sweeps, an A/B build for timing only)
#ifndef SIMAPS_GL_TILE
#define SIMAPS_GL_TILE 1
#endif
bool gl_tiled(int wh, int ww) { return SIMAPS_GL_TILE && (long)gt_tiles(wh, ww) <= GT_MAXT; }

// scratch of the large-window GridGraph kernels (stream-ordered, the library's pool); they have no
// other path, so a launch being captured into a graph is refused instead
int large_scratch(PathScratch &ps, hipStream_t st, size_t bytes, const char *what)
{
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess) return fail(SIMAPS_EHIP, "hipStreamIsCapturing failed");
    if (cap != hipStreamCaptureStatusNone)
        return fail(SIMAPS_EUNSUPPORTED, "%s on a window beyond the LDS-resident limit cannot be captured into a graph "
                    "(its scratch is taken in stream order per launch)", what);
    if (!pool_alloc(ps, st, bytes)) return fail(SIMAPS_EHIP, "%s: no device scratch of %zu bytes", what, bytes);
    return 0;
}


int check_cfg(const simaps_config *c)
{
    if (!c) return fail(SIMAPS_EINVAL, "cfg is NULL");
    if (c->H <= 0 || c->W <= 0 || c->H > 32767 || c->W > 32767) return fail(SIMAPS_EINVAL, "bad grid %dx%d", c->H, c->W);
    if (c->room_h <= 0 || c->room_w <= 0 || c->room_i0 < 0 || c->room_j0 < 0 || c->room_i0 + c->room_h > c->H ||
        c->room_j0 + c->room_w > c->W)
        return fail(SIMAPS_EINVAL, "room rect outside the grid");
    if (c->room_w > SIMAPS_MAX_ROOM_W || c->room_h > MAX_ROWS || (c->room_h + 2) * ((c->room_w + 2) | 1) > SIMAPS_MAX_ROOM_CELLS)
        return fail(SIMAPS_EUNSUPPORTED, "room rect %dx%d exceeds the LDS-resident limit", c->room_h, c->room_w);
    if (c->intention_map_encoding < 0 || c->intention_map_encoding > 3) return fail(SIMAPS_EINVAL, "bad intention encoding");
    if (c->intention_map_line_thickness < 1 || c->intention_map_line_thickness > 2)
        return fail(SIMAPS_EUNSUPPORTED, "intention_map_line_thickness must be 1 or 2");
    if (c->intention_map_scale < 0) return fail(SIMAPS_EUNSUPPORTED, "negative intention_map_scale");
    if (c->rotate_rounding != SIMAPS_ROT_FMA && c->rotate_rounding != SIMAPS_ROT_PLAIN)
        return fail(SIMAPS_EINVAL, "bad rotate_rounding %d", c->rotate_rounding);
    return 0;
}
}  // namespace

extern "C" {

int simaps_abi_version(void) { return SIMAPS_ABI_VERSION; }

#ifndef SIMAPS_SOURCE_HASH  // (the Makefile passes simaps/_srchash.py's digest of the sources)
#define SIMAPS_SOURCE_HASH "unknown"
#endif
const char *simaps_source_hash(void) { return SIMAPS_SOURCE_HASH; }

#if defined(SIMAPS_PHASE_STAMPS) || defined(SIMAPS_LIGHT_STAMPS)
// Diagnostic build only: copy the stamp table (uint64 [8192][NSTAMP]) to host memory.
int simaps_debug_read_stamps(unsigned long long *host_out)
{
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) == hipSuccess ? 0 : SIMAPS_EHIP;
}
#endif

const char *simaps_last_error(void) { return g_err; }

int simaps_fault_status(int clear)
{
    if (!fault_word()) return fail(SIMAPS_EHIP, "could not allocate the host-mapped fault word");
    return (int)read_faults(clear != 0);
}

int simaps_num_channels(const simaps_config *c, int num_robots)
{
    if (!c) return fail(SIMAPS_EINVAL, "cfg is NULL");
    int n = 1 + !!c->use_robot_map + !!c->use_distance_to_receptacle_map + !!c->use_shortest_path_to_receptacle_map +
            !!c->use_shortest_path_map + !!c->use_history_map + !!c->use_intention_map;
    if (c->use_intention_channels) n += (c->intention_channel_spatial ? 1 : 2) * (num_robots - 1);
    return n;
}

int simaps_pack_robots(int R, const double *pose, const double *target, const int32_t *flags, const int32_t *type_group,
                       const double *waypoints, int K, const int32_t *wp_count, const int32_t *wp_index,
                       simaps_robot *robots, double *paths)
{
    if (R < 0 || K < 0) return fail(SIMAPS_EINVAL, "R < 0 or K < 0");
    if (R == 0) return 0;
    if (!pose || !target || !flags || !type_group || !wp_count || !wp_index || !robots || !paths || (K > 0 && !waypoints))
        return fail(SIMAPS_EINVAL, "NULL buffer");
    constexpr int P = SIMAPS_MAX_PATH;
    for (int r = 0; r < R; r++) {
        simaps_robot &o = robots[r];
        const double x = pose[3 * r], y = pose[3 * r + 1];
        const int t = type_group[2 * r], g = type_group[2 * r + 1];
        if (t < 0 || t > 3 || g < 0 || g > 3) return fail(SIMAPS_EINVAL, "robot %d: class %d / group %d", r, t, g);
        const bool idle = flags[r] & 1;
        const int n = wp_count[r], idx = wp_index[r];
        o.x = x;
        o.y = y;
        o.heading = pose[3 * r + 2];
        o.type = t;
        o.group_index = g;
        o.lifting = (flags[r] >> 1) & 1;
        o.idle = idle;
        o.intention_off = 2 * P * r;
        o.history_off = 2 * P * r + P;
        double *ip = paths + (size_t)2 * (2 * P * r), *hp = ip + 2 * P;
        if (n < 0) {  // never acted: waypoints / target / index None (envs.py:828-832, 958-963, 1373-1376)
            if (!idle) return fail(SIMAPS_EINVAL, "robot %d is not idle but has no waypoints", r);
            o.target_x = o.target_y = 0.0;
            o.intention_len = o.history_len = 0;
            continue;
        }
        if (n > K || idx < 0) return fail(SIMAPS_EINVAL, "robot %d: %d waypoints (K = %d), index %d", r, n, K, idx);
        o.target_x = target[2 * r];
        o.target_y = target[2 * r + 1];
        const double *w = waypoints + (size_t)2 * K * r;
        // get_intention_path (envs.py:1475-1476): [position] + waypoints[idx:-1] + [target]
        const int mid = idx < n - 1 ? n - 1 - idx : 0;
        // get_history_path()[::-1] (envs.py:1478-1479, 2318): [position] + waypoints[:idx] reversed
        const int hist = idx < n ? idx : n;
        if (mid + 2 > P || hist + 1 > P) return fail(SIMAPS_EUNSUPPORTED, "robot %d: path longer than %d points", r, P);
        ip[0] = x;
        ip[1] = y;
        for (int k = 0; k < mid; k++) {
            ip[2 + 2 * k] = w[2 * (idx + k)];
            ip[3 + 2 * k] = w[2 * (idx + k) + 1];
        }
        ip[2 + 2 * mid] = target[2 * r];
        ip[3 + 2 * mid] = target[2 * r + 1];
        o.intention_len = mid + 2;
        hp[0] = x;
        hp[1] = y;
        for (int k = 0; k < hist; k++) {
            hp[2 + 2 * k] = w[2 * (hist - 1 - k)];
            hp[3 + 2 * k] = w[2 * (hist - 1 - k) + 1];
        }
        o.history_len = hist + 1;
    }
    return 0;
}

int simaps_robot_mask(int type, int with_cube, float *out)
{
    if (type < 0 || type > 3 || !out) return fail(SIMAPS_EINVAL, "bad robot type / output");
    if (with_cube && type != SIMAPS_LIFTING) return fail(SIMAPS_EINVAL, "lifted cube mask is LiftingRobot only");
    const Geometry &g = geometry();
    for (int i = 0; i < LW; i++)
        for (int j = 0; j < LW; j++) out[i * LW + j] = mask_bit(g, type, with_cube != 0, i, j) ? 1.0f : 0.0f;
    return 0;
}

int simaps_get_state(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                     const simaps_robot *robots, const double *paths, const uint8_t *occupancy, const float *overhead,
                     float *state, int num_robots_per_env, const simaps_debug *dbg, void *stream)
{
    int rc = check_cfg(cfg);
    const Geometry &geo = geometry();
    for (int t = 0; t < 4; t++)
        if (geo.cspace_r[t] > RMAX) return fail(SIMAPS_EUNSUPPORTED, "cspace radius %d > %d", geo.cspace_r[t], RMAX);
    if (rc) return rc;
    if (N < 0) return fail(SIMAPS_EINVAL, "N < 0");
    if (N == 0) return 0;
    if (!agents || !envs || !robots || !occupancy || !overhead || !state) return fail(SIMAPS_EINVAL, "NULL buffer");
    if ((cfg->use_intention_map || cfg->use_history_map) && !paths) return fail(SIMAPS_EINVAL, "paths is NULL");
    if (cfg->use_intention_channels && (num_robots_per_env < 1 || num_robots_per_env > SIMAPS_MAX_ROBOTS))
        return fail(SIMAPS_EINVAL, "intention channels need num_robots_per_env in [1, %d]", SIMAPS_MAX_ROBOTS);
    const int C = simaps_num_channels(cfg, num_robots_per_env > 0 ? num_robots_per_env : 1);
    if ((rc = pending_faults())) return rc;
    simaps_debug d;
    memset(&d, 0, sizeof(d));
    if (dbg) d = *dbg;
#ifdef SIMAPS_VGPR_CAP
    static const hipError_t lds_ok =
        hipFuncSetAttribute((const void *)get_state_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (lds_ok != hipSuccess) return fail(SIMAPS_EHIP, "dynamic LDS of the VGPR-cap build");
    hipLaunchKernelGGL(get_state_kernel, dim3(N), dim3(NT), LDS_BYTES, (hipStream_t)stream, *cfg, geo, agents, envs,
                       robots, paths, occupancy, overhead, state, C, d, g_fault_dev);
#else
    hipLaunchKernelGGL(get_state_kernel, dim3(N), dim3(NT), 0, (hipStream_t)stream, *cfg, geo, agents, envs,
                       robots, paths, occupancy, overhead, state, C, d, g_fault_dev);
#endif
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "get_state launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_get_state_mixed(const simaps_config *cfgs, const int32_t *num_robots_per_env, int n_cfgs, int N,
                           const simaps_agent *agents, const int32_t *agent_cfg, const simaps_env *envs,
                           const simaps_robot *robots, const double *paths, const uint8_t *occupancy,
                           const int64_t *map_off, const float *overhead, float *state, const int64_t *out_off,
                           void *stream)
{
    if (!cfgs || n_cfgs < 1 || n_cfgs > SIMAPS_MAX_MIXED)
        return fail(SIMAPS_EINVAL, "n_cfgs %d not in [1, %d]", n_cfgs, SIMAPS_MAX_MIXED);
    const Geometry &geo = geometry();
    for (int t = 0; t < 4; t++)
        if (geo.cspace_r[t] > RMAX) return fail(SIMAPS_EUNSUPPORTED, "cspace radius %d > %d", geo.cspace_r[t], RMAX);
    simaps_mixed::MixedCfgs mx;
    memset(&mx, 0, sizeof(mx));
    bool any_paths = false;
    for (int k = 0; k < n_cfgs; k++) {
        if (const int rc = check_cfg(&cfgs[k])) return rc;
        const int nr = num_robots_per_env ? num_robots_per_env[k] : 0;
        if (cfgs[k].use_intention_channels && (nr < 1 || nr > SIMAPS_MAX_ROBOTS))
            return fail(SIMAPS_EINVAL, "configuration %d: intention channels need num_robots_per_env in [1, %d]", k,
                        SIMAPS_MAX_ROBOTS);
        mx.cfg[k] = cfgs[k];
        mx.C[k] = simaps_num_channels(&cfgs[k], nr > 0 ? nr : 1);
        any_paths = any_paths || cfgs[k].use_intention_map || cfgs[k].use_history_map;
    }
    mx.n = n_cfgs;
    if (N < 0) return fail(SIMAPS_EINVAL, "N < 0");
    if (N == 0) return 0;
    if (!agents || !agent_cfg || !envs || !robots || !occupancy || !map_off || !overhead || !state || !out_off)
        return fail(SIMAPS_EINVAL, "NULL buffer");
    if (any_paths && !paths) return fail(SIMAPS_EINVAL, "paths is NULL");
    if (const int rc = pending_faults()) return rc;
    simaps_mixed::launch_get_state_mixed(mx, geo, N, agents, agent_cfg, envs, robots, paths, occupancy, map_off, overhead,
                                         state, out_off, g_fault_dev, (hipStream_t)stream);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "get_state_mixed launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_rec_cache_bytes(const simaps_config *cfg)
{
    const int rc = check_cfg(cfg);
    if (rc) return rc;
    return rec_cache_bytes(cfg->room_h, cfg->room_w);
}

int simaps_sp_lookup(const simaps_config *cfg, int N, const simaps_agent *agents, const void *rec_cache,
                     const double *targets, int Q, double *out, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (N < 0 || Q < 0) return fail(SIMAPS_EINVAL, "N < 0 or Q < 0");
    if (N == 0 || Q == 0) return 0;
    if (!agents || !rec_cache || !targets || !out) return fail(SIMAPS_EINVAL, "NULL buffer");
    if ((rc = pending_faults())) return rc;
    hipLaunchKernelGGL(sp_lookup_kernel, dim3(N), dim3(LNT), 0, (hipStream_t)stream, *cfg, agents,
                       reinterpret_cast<const char *>(rec_cache), rec_cache_bytes(cfg->room_h, cfg->room_w), targets, Q, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "sp_lookup launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_sp_distance(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                       const simaps_robot *robots, const uint8_t *occupancy, const double *sources,
                       const double *targets, int Q, double *out, void *rec_cache, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (N < 0 || Q < 0) return fail(SIMAPS_EINVAL, "N < 0 or Q < 0");
    if (N == 0 || Q == 0) return 0;
    if (!agents || !envs || !robots || !occupancy || !sources || !targets || !out)
        return fail(SIMAPS_EINVAL, "NULL buffer");
    if ((rc = pending_faults())) return rc;
    const Geometry &geo = geometry();
    hipLaunchKernelGGL(sp_distance_kernel, dim3(N), dim3(NT), 0, (hipStream_t)stream, *cfg, geo, agents, envs, robots,
                       occupancy, sources, targets, Q, out, reinterpret_cast<char *>(rec_cache), g_fault_dev);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "sp_distance launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_shortest_path(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                         const simaps_robot *robots, const uint8_t *occupancy, const double *sources,
                         const double *targets, int max_points, double *out_xy, int32_t *out_count, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (N < 0 || max_points < 2) return fail(SIMAPS_EINVAL, "N < 0 or max_points < 2");
    if (N == 0) return 0;
    if (!agents || !envs || !robots || !occupancy || !sources || !targets || !out_xy || !out_count)
        return fail(SIMAPS_EINVAL, "NULL buffer");
    if ((rc = pending_faults())) return rc;
    const Geometry &geo = geometry();
    const bool small = (cfg->room_h + 2) * ((cfg->room_w + 2) | 1) <= PATH_SMALL_CELLS;
    const hipStream_t st = (hipStream_t)stream;
    const PathKind kind = path_kind(N, small);
    PathScratch ps;
    if (kind == PK_EARLY) path_scratch(ps, st, (size_t)N * SIMAPS_MAX_ROOM_CELLS * sizeof(float));
    float *scratch = ps.p;
#define SIMAPS_PATH_LAUNCH(C, E, O)                                                                    \
    hipLaunchKernelGGL((path_kernel<C, E, O>), dim3(N), dim3(PNT), 0, st, *cfg, geo, agents, envs, robots, occupancy, \
                       sources, targets, max_points, out_xy, out_count, scratch, g_fault_dev)
    if (kind == PK_OVL) {
        if (small) SIMAPS_PATH_LAUNCH(PATH_SMALL_CELLS, true, true);
        else SIMAPS_PATH_LAUNCH(SIMAPS_MAX_ROOM_CELLS, true, true);
    } else if (scratch) {
        if (small) SIMAPS_PATH_LAUNCH(PATH_SMALL_CELLS, true, false);
        else SIMAPS_PATH_LAUNCH(SIMAPS_MAX_ROOM_CELLS, true, false);
    } else {
        if (small) SIMAPS_PATH_LAUNCH(PATH_SMALL_CELLS, false, false);
        else SIMAPS_PATH_LAUNCH(SIMAPS_MAX_ROOM_CELLS, false, false);
    }
#undef SIMAPS_PATH_LAUNCH
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "shortest_path launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_path_mode(int mode)
{
    if (mode < 0 || mode > 3) return fail(SIMAPS_EINVAL, "path mode %d not in 0..3", mode);
    return g_path_mode.exchange(mode);
}

int simaps_ingest_chunks(int height_px, int width_px)
{
    if (height_px <= 0 || width_px <= 0) return fail(SIMAPS_EINVAL, "bad camera size");
    return ingest_chunks(height_px, width_px);
}

int simaps_ingest(const simaps_config *cfg, const simaps_camera *cam, int N, const simaps_agent *agents,
                  const simaps_seg_ids *seg_ids, const double *cam_params, const float *depth, const int32_t *seg_raw,
                  float *overhead, uint8_t *occupancy, uint64_t *keys, uint32_t *boxes, int epoch, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (!cam || cam->height_px <= 0 || cam->width_px <= 0 || !(cam->far_m > cam->near_m) || !(cam->near_m > 0))
        return fail(SIMAPS_EINVAL, "bad camera");
    if (N < 0) return fail(SIMAPS_EINVAL, "N < 0");
    if (N == 0) return 0;
    if (!agents || !seg_ids || !cam_params || !depth || !seg_raw || !overhead || !occupancy || !keys || !boxes)
        return fail(SIMAPS_EINVAL, "NULL buffer");
    const int np = cam->height_px * cam->width_px;
    if (!ingest_width_ok(cam->width_px))
        return fail(SIMAPS_EUNSUPPORTED, "camera width %d outside [%d, %d]", cam->width_px, ingest_min_width(), INGEST_MAX_WC);
    if (np >= (1 << 20)) return fail(SIMAPS_EUNSUPPORTED, "camera frame of %d pixels (key packs pixel + 1 in 20 bits)", np);
    if (epoch < 0 || epoch > 255) return fail(SIMAPS_EINVAL, "epoch %d not in [0, 255]", epoch);
    {   // a captured launch replays its epoch: only the zeroing mode (epoch 0) leaves nothing behind
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess)
            return fail(SIMAPS_EHIP, "hipStreamIsCapturing failed");
        if (cap != hipStreamCaptureStatusNone && epoch != 0)
            return fail(SIMAPS_EUNSUPPORTED, "ingest with epoch %d under stream capture: every replay would reuse "
                        "the epoch; pass epoch 0 (zeroing mode) on an all-zero key map", epoch);
    }
    const bool zero_mode = epoch == 0;
    if (zero_mode) epoch = 1;
    if (N > 65535) return fail(SIMAPS_EUNSUPPORTED, "%d frames per launch (grid y <= 65535)", N);
    const int nch = ingest_chunks(cam->height_px, cam->width_px);  // point-pass chunks per frame
    if ((rc = pending_faults())) return rc;  // (after the argument checks: they need no device)
    if (cam->width_px + INGEST_PPT <= 320)
        hipLaunchKernelGGL(ingest_points_kernel<320>, dim3(nch, N), dim3(INGEST_WG), 0, (hipStream_t)stream, *cfg, *cam, agents,
                           seg_ids, cam_params, depth, seg_raw, occupancy, reinterpret_cast<unsigned long long *>(keys), boxes, (unsigned)epoch);
    else
        hipLaunchKernelGGL(ingest_points_kernel<INGEST_MAX_WC>, dim3(nch, N), dim3(INGEST_WG), 0, (hipStream_t)stream, *cfg, *cam,
                           agents, seg_ids, cam_params, depth, seg_raw, occupancy, reinterpret_cast<unsigned long long *>(keys), boxes, (unsigned)epoch);
    if (zero_mode)
        hipLaunchKernelGGL(ingest_resolve_kernel<true>, dim3(INGEST_RES_G, N), dim3(INGEST_RES_WG), 0, (hipStream_t)stream, *cfg,
                           agents, overhead, reinterpret_cast<unsigned long long *>(keys), boxes, nch, (unsigned)epoch);
    else
        hipLaunchKernelGGL(ingest_resolve_kernel<false>, dim3(INGEST_RES_G, N), dim3(INGEST_RES_WG), 0, (hipStream_t)stream, *cfg,
                           agents, overhead, reinterpret_cast<unsigned long long *>(keys), boxes, nch, (unsigned)epoch);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "ingest launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_grid_path(int B, int H, int W, const uint8_t *grids, const int32_t *sources, const int32_t *targets,
                     int wi0, int wj0, int wh, int ww, int max_points, int32_t *out_ij, int32_t *out_count, void *stream)
{
    if (B < 0 || H <= 0 || W <= 0 || max_points < 1) return fail(SIMAPS_EINVAL, "bad batch / grid shape / max_points");
    if (H > 32767 || W > 32767) return fail(SIMAPS_EINVAL, "grid %dx%d too large", H, W);
    if (B == 0) return 0;
    if (!grids || !sources || !targets || !out_ij || !out_count) return fail(SIMAPS_EINVAL, "NULL buffer");
    if (wh <= 0 || ww <= 0 || wi0 < 0 || wj0 < 0 || wi0 + wh > H || wj0 + ww > W)
        return fail(SIMAPS_EINVAL, "window outside the grid");
    const hipStream_t st = (hipStream_t)stream;
    if (!window_fits_lds(wh, ww)) {  // any larger window: the global-memory kernels (grid_large.h)
        if (const int rc = pending_faults()) return rc;
        const long words = gl_path_words(wh, ww);
        PathScratch ps;
        if (const int rc = large_scratch(ps, st, (size_t)B * words * sizeof(int), "grid_path")) return rc;
        if (gl_tiled(wh, ww))
            hipLaunchKernelGGL(gl_tile_kernel, dim3(B), dim3(GT_NT), 0, st, H, W, grids, (long)H * W, sources, wi0, wj0, wh,
                               ww, ps.p, words, nullptr, g_fault_dev);
        else
            hipLaunchKernelGGL(gl_sssp_kernel, dim3(B), dim3(GL_NT), 0, st, H, W, grids, (long)H * W, sources, wi0, wj0, wh,
                               ww, ps.p, words, nullptr, g_fault_dev);
        hipLaunchKernelGGL(gl_path_kernel, dim3(B), dim3(64), 0, st, H, W, grids, (long)H * W, sources, targets, wi0, wj0,
                           wh, ww, reinterpret_cast<int *>(ps.p), words, max_points, out_ij, out_count, g_fault_dev);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(SIMAPS_EHIP, "grid_path (large window) launch: %s", hipGetErrorString(e));
        return 0;
    }
    if (const int rc = pending_faults()) return rc;
    const bool small = (wh + 2) * ((ww + 2) | 1) <= PATH_SMALL_CELLS;
    const PathKind kind = path_kind(B, small);
    PathScratch ps;
    if (kind == PK_EARLY) path_scratch(ps, st, (size_t)B * SIMAPS_MAX_ROOM_CELLS * sizeof(float));
    float *scratch = ps.p;
#define SIMAPS_GRID_PATH_LAUNCH(C, E, O)                                                               \
    hipLaunchKernelGGL((grid_path_kernel<C, E, O>), dim3(B), dim3(PNT), 0, st, H, W, grids, sources, targets, wi0, wj0, \
                       wh, ww, max_points, out_ij, out_count, scratch, g_fault_dev)
    if (kind == PK_OVL) {
        if (small) SIMAPS_GRID_PATH_LAUNCH(PATH_SMALL_CELLS, true, true);
        else SIMAPS_GRID_PATH_LAUNCH(SIMAPS_MAX_ROOM_CELLS, true, true);
    } else if (scratch) {
        if (small) SIMAPS_GRID_PATH_LAUNCH(PATH_SMALL_CELLS, true, false);
        else SIMAPS_GRID_PATH_LAUNCH(SIMAPS_MAX_ROOM_CELLS, true, false);
    } else {
        if (small) SIMAPS_GRID_PATH_LAUNCH(PATH_SMALL_CELLS, false, false);
        else SIMAPS_GRID_PATH_LAUNCH(SIMAPS_MAX_ROOM_CELLS, false, false);
    }
#undef SIMAPS_GRID_PATH_LAUNCH
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "grid_path launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_sssp_grid(int B, int H, int W, const uint8_t *grids, const int32_t *sources, float *dists, int wi0, int wj0,
                     int wh, int ww, void *stream)
{
    if (B < 0 || H <= 0 || W <= 0) return fail(SIMAPS_EINVAL, "bad batch / grid shape");
    if (B == 0) return 0;
    if (!grids || !sources || !dists) return fail(SIMAPS_EINVAL, "NULL buffer");
    if (wh <= 0 || ww <= 0 || wi0 < 0 || wj0 < 0 || wi0 + wh > H || wj0 + ww > W)
        return fail(SIMAPS_EINVAL, "window outside the grid");
    if (H > 32767 || W > 32767) return fail(SIMAPS_EINVAL, "grid %dx%d too large", H, W);
    if (!window_fits_lds(wh, ww)) {  // any larger window: the global-memory sweeps (grid_large.h)
        if (const int rc = pending_faults()) return rc;
        const hipStream_t st = (hipStream_t)stream;
        const long cells = (long)(wh + 2) * (ww + 2);
        PathScratch ps;
        if (const int rc = large_scratch(ps, st, (size_t)B * cells * sizeof(float), "sssp_grid")) return rc;
        if (gl_tiled(wh, ww))
            hipLaunchKernelGGL(gl_tile_kernel, dim3(B), dim3(GT_NT), 0, st, H, W, grids, (long)H * W, sources, wi0, wj0, wh,
                               ww, ps.p, cells, dists, g_fault_dev);
        else
            hipLaunchKernelGGL(gl_sssp_kernel, dim3(B), dim3(GL_NT), 0, st, H, W, grids, (long)H * W, sources, wi0, wj0, wh,
                               ww, ps.p, cells, dists, g_fault_dev);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(SIMAPS_EHIP, "sssp_grid (large window) launch: %s", hipGetErrorString(e));
        return 0;
    }
    if (const int rc = pending_faults()) return rc;
    hipLaunchKernelGGL(sssp_grid_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, H, W, grids, sources, dists, wi0,
                       wj0, wh, ww, g_fault_dev);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "sssp_grid launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_occupancy_scatter(const simaps_config *cfg, int N, const simaps_agent *agents, const float *points,
                             const float *seg, int P, double obstacle_seg_value, uint8_t *occupancy, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (N < 0 || P < 0) return fail(SIMAPS_EINVAL, "N < 0 or P < 0");
    if (N == 0 || P == 0) return 0;
    if (!agents || !points || !seg || !occupancy) return fail(SIMAPS_EINVAL, "NULL buffer");
    if (N > 65535) return fail(SIMAPS_EUNSUPPORTED, "%d maps per launch (grid y <= 65535)", N);
    if ((rc = pending_faults())) return rc;
    hipLaunchKernelGGL(occupancy_scatter_kernel, dim3((P + 255) / 256, N), dim3(256), 0, (hipStream_t)stream, cfg->H,
                       cfg->W, P, agents, points, seg, obstacle_seg_value, occupancy);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "occupancy_scatter launch: %s", hipGetErrorString(e));
    return 0;
}

static int occupancy_map_launch(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                         const simaps_robot *robots, const uint8_t *occupancy, uint8_t *cspace, uint8_t *thin,
                         const int32_t *pixels, int Q, int32_t *snapped, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (N < 0 || Q < 0) return fail(SIMAPS_EINVAL, "N < 0 or Q < 0");
    if (N == 0) return 0;
    if (!agents || !envs || !robots || !occupancy) return fail(SIMAPS_EINVAL, "NULL buffer");
    if (N > 65535) return fail(SIMAPS_EUNSUPPORTED, "%d agents per launch (grid y <= 65535)", N);
    if ((rc = pending_faults())) return rc;
    const int chunks = snapped ? (Q + OCC_SNAP_PER_WG - 1) / OCC_SNAP_PER_WG : 1;
    if (chunks == 0) return 0;
    hipLaunchKernelGGL(occupancy_map_kernel, dim3(chunks, N), dim3(PNT), 0, (hipStream_t)stream, *cfg, geometry(), agents,
                       envs, robots, occupancy, cspace, thin, pixels, Q, snapped, g_fault_dev);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "occupancy_map launch: %s", hipGetErrorString(e));
    return 0;
}

int simaps_build_cspace(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                        const simaps_robot *robots, const uint8_t *occupancy, uint8_t *cspace, uint8_t *cspace_thin,
                        void *stream)
{
    if (!cspace && !cspace_thin) return fail(SIMAPS_EINVAL, "neither cspace nor cspace_thin requested");
    return occupancy_map_launch(cfg, N, agents, envs, robots, occupancy, cspace, cspace_thin, nullptr, 0, nullptr, stream);
}

int simaps_snap_sources(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                        const simaps_robot *robots, const uint8_t *occupancy, const int32_t *pixels, int Q,
                        int32_t *out, void *stream)
{
    if (Q > 0 && (!pixels || !out)) return fail(SIMAPS_EINVAL, "NULL buffer");
    if (Q == 0) return 0;
    return occupancy_map_launch(cfg, N, agents, envs, robots, occupancy, nullptr, nullptr, pixels, Q, out, stream);
}

int simaps_global_maps(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                       const simaps_robot *robots, const double *paths, const float *overhead, float *overhead_map,
                       float *robot_map, float *history_map, float *intention_map, void *stream)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (N < 0) return fail(SIMAPS_EINVAL, "N < 0");
    if (N == 0 || (!overhead_map && !robot_map && !history_map && !intention_map)) return 0;
    if (!agents || !envs || !robots || !paths || (overhead_map && !overhead)) return fail(SIMAPS_EINVAL, "NULL buffer");
    if ((rc = pending_faults())) return rc;
    hipLaunchKernelGGL(global_maps_kernel, dim3(N), dim3(NT), 0, (hipStream_t)stream, *cfg, geometry(), agents, envs,
                       robots, paths, overhead, overhead_map, robot_map, history_map, intention_map, g_fault_dev);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SIMAPS_EHIP, "global_maps launch: %s", hipGetErrorString(e));
    return 0;
}

}  // extern "C"
#endif  // SIMAPS_DEVICE_ONLY
