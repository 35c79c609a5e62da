// GridGraph on grids whose free cells span more than the LDS-resident window (include/simaps.h
// SIMAPS_MAX_ROOM_CELLS / SIMAPS_MAX_ROOM_W): the reference's GridGraph(grid) takes any C-contiguous
// uint8 grid (shortest_paths.pyx:24-38).  Included by simaps.hip inside its device namespace; the
// C ABI (simaps_sssp_grid / simaps_grid_path) dispatches here when a window does not fit.
//
// Same algorithm as the LDS kernels, with the arrays in global memory (L2-resident for grids up to a
// few Mcells) and one workgroup per query:
//   gl_tile_kernel  (round 6, windows of up to GT_MAXT tiles) the same fixpoint through 62 x 62-cell LDS
//                   tiles taken from a queue of dirty tiles by four 4-wave groups (below)
//   gl_sssp_kernel  (larger windows) the float32 fixpoint by directional sweeps (down / up / right / left, GL_WPD waves
//                   each over 64-cell strips of their lines, lines prefetched ahead); every write is
//                   an atomic min(cell, fl(d_u + w)) of a real edge, so the unique fixpoint -- the
//                   reference SPFA's distances (pyx:69-114), bit for bit -- is reached whatever the
//                   interleaving, and a round in which no sweep finds a candidate below the value it
//                   read proves it (values only fall; in a round without writes every read is exact).
//   gl_path_kernel  one wave per query: the exact SPFA replay (edge order, SLF swap, pyx:89-107) with
//                   the early exit of the LDS kernels (it stops once every vertex of the target's
//                   parent chain holds its fixpoint distance: no parent on it can change any more;
//                   checked every 64 pops, resuming the chain walk where it stopped),
//                   the parent walk, approximate_polygon(tolerance=1) and the line-of-sight pruning
//                   (pyx:121-154).  The SPFA is serial by definition: one round of loads per pop.
// Padded layout per query: (wh + 2) rows x pitch = ww + 2 columns, border and blocked cells -inf,
// free cells +inf until reached.

#ifndef SIMAPS_GL_WPD
#define SIMAPS_GL_WPD 1
#endif
constexpr int GL_WPD = SIMAPS_GL_WPD;  // gl_sssp_kernel: waves per sweep direction (each takes every
constexpr int GL_NT = 4 * 64 * GL_WPD;  //  GL_WPD-th 64-cell strip of its direction's lines)
#ifndef SIMAPS_GL_PF
#define SIMAPS_GL_PF 32
#endif
constexpr int GL_PF = SIMAPS_GL_PF;  // lines prefetched ahead in a sweep strip
constexpr int GL_INQ = 16;  // pin bit 4: in the queue (bits 0-3: 1 + direction of the parent edge)
constexpr int GL_CHECK = 64;  // gl_path_kernel: pops between early-exit checks

struct GlDims {
    int wh, ww, pitch;
    long cells;
};

__device__ __forceinline__ GlDims gl_dims(int wh, int ww) { return GlDims{wh, ww, ww + 2, (long)(wh + 2) * (ww + 2)}; }

// Loads that see what other waves (and lanes) of the workgroup wrote through L2: agent scope (the
// vector L1 is not coherent with the atomics / stores of other waves).
__device__ __forceinline__ float gl_ld(const float *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int gl_ldi(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gl_st(float *p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gl_sti(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// every store / atomic of this wave has reached L2 before the next load issues
__device__ __forceinline__ void gl_drain() { __builtin_amdgcn_s_waitcnt(0); }

// lane k's value (k wave-uniform) in every lane
__device__ __forceinline__ int gl_lane(int x, int k) { return __builtin_amdgcn_readlane(x, k); }
__device__ __forceinline__ float gl_lane(float x, int k) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), k)); }

// lane i <- lane i - 1 (lane 0 <- edge) / lane i <- lane i + 1 (lane 63 <- edge): DPP wave_shr:1 /
// wave_shl:1 with bound_ctrl off, so the lane without a source keeps the `old` operand
__device__ __forceinline__ float gl_from_prev_lane(float v, float edge)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float gl_from_next_lane(float v, float edge)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x130, 0xf, 0xf, false));
}

// One sweep of one wave over every line of the window (DIR 0 down, 1 up: lines = rows; 2 right,
// 3 left: lines = columns), 64 cells of each line at a time (strip s0).  A cell of line l is relaxed
// from the 3 cells of line l -1 (in sweep order): straight (weight 1) and the two diagonals (float32
// sqrt(2)).  Inside a strip the previous line's values pass between lanes by DPP; lane 0 / lane 63
// read their outer neighbour from memory (the neighbouring strip's value, as far as its wave got in
// this sweep or from before it) -- a stale value is still some path's length, so every write remains
// a valid relaxation.  Returns true if some candidate was below the value read.
template <int DIR>
__device__ bool gl_sweep(float *D, const GlDims g, int part)
{
    constexpr bool VERT = DIR < 2, FWD = (DIR & 1) == 0;
    const int lane = threadIdx.x & 63;
    const int N = VERT ? g.wh : g.ww, L = VERT ? g.ww : g.wh;
    const int sl = VERT ? g.pitch : 1, sa = VERT ? 1 : g.pitch;
    bool chg = false;
    // Plain loads through the L1, addressed as a wave-uniform line pointer (SGPRs) plus a 32-bit
    // per-lane offset: a line the L1 still holds from before another wave's atomics is stale, which
    // is allowed (see above); gl_sssp_kernel invalidates the L1 at every round's barrier, so in a
    // round without writes every read is current.
    auto line = [&](int t) { return D + (long)((FWD ? 1 + t : N - t) * sl); };
    for (int s0 = 64 * part; s0 < L; s0 += 64 * GL_WPD) {
        const int c = s0 + lane;
        const bool act = c < L;
        const int cc = act ? c : L;  // inactive lanes alias the border cell after the line (-inf)
        const int own = (1 + cc) * sa;
        // the outer neighbour a strip edge reads (lane 0: c - 1, lane 63: c + 1); others re-read their own cell
        const int xo = (1 + (lane == 0 ? c - 1 : (lane == 63 && act) ? c + 1 : cc)) * sa;
        const float one = act ? 1.0f : INFINITY, s2 = act ? SQRT2F : INFINITY;
        float Rr[GL_PF], Xr[GL_PF];
#pragma unroll
        for (int j = 0; j < GL_PF; j++)
            if (j < N) {
                const float *ln = line(j);
                Rr[j] = ln[own];
                Xr[j] = ln[xo];
            }
        // the previous line: this lane's value (sign trick: -inf = blocked passes on nothing, as |.|
        // = +inf) and its outer neighbour's
        float p = INFINITY, xp = INFINITY;
        for (int t0 = 0; t0 < N; t0 += GL_PF) {
#pragma unroll
            for (int j = 0; j < GL_PF; j++) {
                const int t = t0 + j;
                if (t < N) {  // (wave-uniform)
                    const float R = Rr[j], X = Xr[j];
                    if (t + GL_PF < N) {
                        const float *ln = line(t + GL_PF);
                        Rr[j] = ln[own];
                        Xr[j] = ln[xo];
                    }
                    // wave shifts with the strip edge's own neighbour as the `old` value of lane 0 /
                    // lane 63 (no select: a select became a branch around the DPP move, and a DPP read
                    // from a lane that branch had disabled returns 0 -- a fake neighbour at distance 0)
                    const float pl = gl_from_prev_lane(p, xp);
                    const float pr = gl_from_next_lane(p, xp);
                    const float m = fminf(fminf(fabsf(p) + one, fabsf(pl) + s2), fabsf(pr) + s2);
                    if (m < R) {  // (blocked / border cells hold -inf: never)
                        atomicMin(reinterpret_cast<int *>(line(t)) + own, __float_as_int(m));  // m >= 0: int order
                        chg = true;
                    }
                    p = act ? fminf(m, R) : -INFINITY;
                    xp = X;
                }
            }
        }
    }
    return __ballot(chg) != 0;
}

// Batched GridGraph(grid).shortest_path_image(source) for windows of any size.  scratch: one padded
// array per query (the fixpoint: gl_path_kernel's early-exit reference); out (may be null): the
// [H, W] image as pyx:110-112 leaves it (-1 unreachable, 0 at the source even when blocked).
__global__ void __launch_bounds__(GL_NT) gl_sssp_kernel(int H, int W, const uint8_t *__restrict__ grids, long grid_stride,
                                                       const int32_t *__restrict__ sources, int wi0, int wj0, int wh, int ww,
                                                       float *scratch, long scratch_stride, float *__restrict__ out,
                                                       unsigned *fault)
{
    __shared__ int changed[3];
    const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6;
    const uint8_t *grid = grids + b * grid_stride;
    const GlDims g = gl_dims(wh, ww);
    float *D = scratch + b * scratch_stride;
    const int si = sources[2 * b], sj = sources[2 * b + 1];
    const bool s_in = si >= wi0 && si < wi0 + wh && sj >= wj0 && sj < wj0 + ww && grid[(long)si * W + sj] != 0;
    const long sq = s_in ? (long)(si - wi0 + 1) * g.pitch + (sj - wj0 + 1) : -1;
    for (long k = tid; k < g.cells; k += GL_NT) {
        const int r = (int)(k / g.pitch), c = (int)(k - (long)r * g.pitch);
        float v = -INFINITY;
        if (r >= 1 && r <= wh && c >= 1 && c <= ww && grid[(long)(wi0 + r - 1) * W + wj0 + c - 1] != 0)
            v = k == sq ? 0.0f : INFINITY;
        gl_st(D + k, v);
    }
    if (tid < 3) changed[tid] = 0;
    gl_drain();
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    unsigned f = 0;
    if (s_in) {
        const long cap = (long)wh * ww + 16;
        for (long round = 0;; round++) {
            const int dir = wave & 3, part = wave >> 2;  // (strips of one direction run side by side)
            const bool c = dir == 0 ? gl_sweep<0>(D, g, part) : dir == 1 ? gl_sweep<1>(D, g, part)
                         : dir == 2 ? gl_sweep<2>(D, g, part) : gl_sweep<3>(D, g, part);
            if (c && (tid & 63) == 0) changed[round % 3] = 1;
            if (tid == 0) changed[(round + 1) % 3] = 0;  // (last read two barriers ago)
            gl_drain();  // this round's atomics are in L2 before any wave reads for the next one
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (invalidates the L1: the next round reads L2)
            if (!changed[round % 3]) break;
            if (round >= cap) {
                f = SIMAPS_FAULT_ROUNDS;
                break;
            }
        }
    }
    if (tid == 0) post_faults(fault, f);
    if (!out) return;
    float *o = out + (long)b * H * W;
    for (long k = tid; k < (long)H * W; k += GL_NT) {
        const int i = (int)(k / W), j = (int)(k - (long)i * W);
        float v = (i == si && j == sj) ? 0.0f : -1.0f;
        const int r = i - wi0, c = j - wj0;
        if (r >= 0 && r < wh && c >= 0 && c < ww) {
            const float d = gl_ld(D + (long)(r + 1) * g.pitch + c + 1);
            if (d >= 0.0f && d != INFINITY) v = d;
        }
        o[k] = v;
    }
}

// ---- the tiled fixpoint (round 6) ----------------------------------------------------------------
// gl_sssp_kernel's four waves sweep the WHOLE window every round (a 500 x 500 window: ~20 rounds of
// 4 x 250 k cell-steps from global memory, 7 ms).  gl_tile_kernel does the same fixpoint with work
// only where values still fall: the padded array stays in global memory (L2), cut into GT_TT x GT_TT
// tiles; four groups of four waves take dirty tiles from an LDS queue.  A group loads its tile with a
// one-cell halo into LDS, relaxes the tile's edge cells from the halo (which it only reads), sweeps
// the interior down / up / right / left (sweep_t, one wave per direction) until a round changes
// nothing, writes back the cells that fell and marks the neighbour tiles whose halo they are.  Every
// value written is some path's left-fold float32 length (a stale halo value included), so the
// unique fixpoint -- the reference SPFA's distances (pyx:69-114), bit for bit -- is reached when the
// queue is empty and no group is busy: every edge inside a tile was relaxed by its last processing,
// every edge into it from a halo cell after that cell's last change (which marked the tile).  A
// tile is never processed by two groups at once (a mark that finds it busy asks its group to run it
// again), so write-back is a plain store.  Host model, bitwise against the oracle with tile counts:
// tools/tile_sssp_model.py (~2.3 processings per tile, ~2.2 sweep rounds per processing on 500^2).
constexpr int GT_TT = 62;                       // tile interior side: one cell per lane (span <= 63)
constexpr int GT_TP = 65;                       // LDS pitch of a tile buffer (odd: column sweeps spread over banks)
constexpr int GT_PAD = 8;                       // rows of slack around a buffer (sweep_t's prefetch reads up to
                                                //  6 lines past either end of the tile)
constexpr int GT_BUF = (GT_TT + 2 + 2 * GT_PAD) * GT_TP;  // floats per group buffer
constexpr int GT_GROUPS = 4;
constexpr int GT_NT = 256 * GT_GROUPS;
constexpr int GT_MAXT = 4096;                   // tiles per window (larger windows: gl_sssp_kernel)
constexpr unsigned GT_Q = 1, GT_BUSY = 2, GT_AGAIN = 4;  // tile states (one byte per tile)
constexpr unsigned GT_EMPTY = 0xffffffffu;      // a free ring slot
struct GtShared {
    unsigned bar[GT_GROUPS][4];                 // the groups' LDS barriers (Group)
    unsigned st[GT_MAXT / 4];                   // tile state bytes
    unsigned ring[GT_MAXT];                     // queue of dirty tiles (each at most once)
    unsigned head, tail, outstanding, processed, abort;
    int gtile[GT_GROUPS];                       // the tile a group works on next (-1: done)
    unsigned chg[GT_GROUPS][3];                 // per group, per round: a sweep lowered a cell
    unsigned emask[GT_GROUPS];                  // per group: which edges / corners of its tile fell
    uint64_t gdm[GT_GROUPS][4];                 // per group and sweep direction: lines to relax out of
};                                              //  again (bit L - 1 = line L; a tile has <= 62 lines)
__host__ __device__ constexpr int gt_tiles(int wh, int ww) { return ((wh + GT_TT - 1) / GT_TT) * ((ww + GT_TT - 1) / GT_TT); }

__device__ __forceinline__ unsigned gt_lds_ld(const unsigned *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// a tile's state byte: CAS on its word; f(old byte) -> new byte, or -1 to leave it.  Returns the old byte.
template <class F>
__device__ __forceinline__ unsigned gt_state(GtShared &sh, int t, F f)
{
    unsigned *w = &sh.st[t >> 2];
    const int s8 = (t & 3) * 8;
    unsigned old = gt_lds_ld(w);
    for (;;) {
        const unsigned s = (old >> s8) & 0xffu;
        const int ns = f(s);
        if (ns < 0) return s;
        const unsigned nw = (old & ~(0xffu << s8)) | ((unsigned)ns << s8);
        const unsigned prev = atomicCAS(w, old, nw);
        if (prev == old) return s;
        old = prev;
    }
}

// the tile's halo changed: queue it, or have its busy group run it again
__device__ __forceinline__ void gt_mark(GtShared &sh, int t, int nt)
{
    const unsigned s = gt_state(sh, t, [](unsigned s) -> int {
        if (s & GT_BUSY) return (s & GT_AGAIN) ? -1 : (int)(s | GT_AGAIN);
        return (s & GT_Q) ? -1 : (int)(s | GT_Q);
    });
    if ((s & (GT_BUSY | GT_Q)) == 0) {  // this call queued it
        atomicAdd(&sh.outstanding, 1u);
        const unsigned k = atomicAdd(&sh.tail, 1u) % (unsigned)nt;
        unsigned spins = 0;  // (the slot's previous entry may still be being taken: live entries <= nt)
        while (atomicCAS(&sh.ring[k], GT_EMPTY, (unsigned)t) != GT_EMPTY)
            if (++spins > (1u << 22)) { __hip_atomic_store(&sh.abort, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); break; }
    }
}

// next dirty tile (busy from now on), or -1 when the queue is empty and no group is busy (or on abort)
__device__ __forceinline__ int gt_pop(GtShared &sh, int nt)
{
    unsigned spins = 0;
    for (;;) {
        if (gt_lds_ld(&sh.abort)) return -1;
        const unsigned h = gt_lds_ld(&sh.head);
        if (h != gt_lds_ld(&sh.tail)) {
            if (atomicCAS(&sh.head, h, h + 1) != h) continue;
            unsigned v;
            while ((v = atomicExch(&sh.ring[h % (unsigned)nt], GT_EMPTY)) == GT_EMPTY)  // (its push is landing)
                if (++spins > (1u << 22)) { __hip_atomic_store(&sh.abort, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); return -1; }
            gt_state(sh, (int)v, [](unsigned s) -> int { return (int)((s & ~GT_Q) | GT_BUSY); });
            return (int)v;
        }
        if (gt_lds_ld(&sh.outstanding) == 0) return -1;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { __hip_atomic_store(&sh.abort, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); return -1; }
    }
}

// the group finished tile t: true if it must run it again (marked while busy)
__device__ __forceinline__ bool gt_finish(GtShared &sh, int t)
{
    const unsigned s = gt_state(sh, t, [](unsigned s) -> int { return (s & GT_AGAIN) ? (int)(s & ~GT_AGAIN) : (int)(s & ~GT_BUSY); });
    if (s & GT_AGAIN) return true;
    atomicSub(&sh.outstanding, 1u);
    return false;
}

// One directional sweep of the tile's interior over its dirty lines only: the get_state kernels'
// dirty-line rule (simaps.hip sweep()) with the inline-asm step loop at the tile pitch.  The wave
// snapshot-clears its direction's mask, sweeps from the first dirty line and stops at the first
// non-improving group of 4 lines past the last one; it marks the lines it lowered for the opposite
// direction and the lines of its improving lanes for the two perpendicular ones.  Marks follow the
// sweep's own writes (the asm drains them) and the snapshot precedes its reads, so a decrease is
// either seen or left marked; a round without improvement leaves every mask empty = the tile's local
// fixpoint.  A tile's first lines to sweep are those of the edge cells its halo lowered (and the
// source's), so a small halo change costs a small sweep.  (Whole sweeps with sweep_t: 1.05 ms per
// 500^2 image, r6x.)
template <int DIR>
__device__ __forceinline__ bool gt_sweep(lds_float *L, int th, int tw, uint64_t *dm)
{
    constexpr bool VERT = DIR < 2, FWD = (DIR & 1) == 0;
    const int len = VERT ? th : tw, span = VERT ? tw : th;
    uint64_t m = 0;
    if ((threadIdx.x & 63) == 0) m = __hip_atomic_exchange(&dm[DIR], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(m >> 32)) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
    if (!m) return false;
    const int blo = __builtin_ctzll(m), bhi = 63 - __builtin_clzll(m);
    const int t0 = FWD ? blo : len - 1 - bhi, tmax = FWD ? bhi : len - 1 - blo;  // step t: line FWD ? t + 1 : len - t
    const SweepOut o = sweep_asm<DIR, 1, GT_TP>(L, len, span, t0, tmax, len);
    if (!o.lanes) return false;
    if ((threadIdx.x & 63) == 0) {
        const int a = FWD ? o.imin : len - 1 - o.imax, b = FWD ? o.imax : len - 1 - o.imin;
        __hip_atomic_fetch_or(&dm[DIR ^ 1], bits64(max(a, 0), min(b, 63)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        constexpr int P = VERT ? 2 : 0;  // lane i owns line i + 1 of the perpendicular directions
        __hip_atomic_fetch_or(&dm[P], o.lanes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(&dm[P + 1], o.lanes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return true;
}

// a changed cell (row a, column b of the tile, 1-based) dirties its row for the vertical sweeps and its
// column for the horizontal ones
__device__ __forceinline__ void gt_mark_lines(uint64_t *dm, int a, int b)
{
    __hip_atomic_fetch_or(&dm[0], 1ull << (a - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&dm[1], 1ull << (a - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&dm[2], 1ull << (b - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&dm[3], 1ull << (b - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One group's processing of tile (ti, tj): load with halo -> edge relaxation -> sweep rounds -> write-back.
// Returns the edge mask (bits: top, bottom, left, right rows / columns; corners (1,1), (1,tw), (th,1),
// (th,tw)) of the cells that fell, in the group's leader; every thread of the group calls it.
__device__ __forceinline__ unsigned gt_process(GtShared &sh, lds_float *L, float *D, const GlDims g, int ti, int tj,
                                               const Group &grp, int gi, int sr, int sc)
{
    const int t = grp.t, dir = t >> 6;
    const int r0 = ti * GT_TT, c0 = tj * GT_TT;
    const int th = min(GT_TT, g.wh - r0), tw = min(GT_TT, g.ww - c0);
    // Padded rows r0 .. r0 + th + 1, columns c0 .. c0 + tw + 1 (the halo: the neighbours' edge cells or
    // the -inf border): wave w of the group takes rows w, w + 4, .., lane = column.  All 16 loads of a
    // lane go out together (addresses clamped into the tile, so none is masked); the values stay in
    // registers for the write-back's comparison.
    const int lane = t & 63, a0 = t >> 6;
    const int lb = min(lane, tw + 1);
    const float *src = D + (long)r0 * g.pitch + c0 + lb;
    float old[16];
#pragma unroll
    for (int j = 0; j < 16; j++) old[j] = gl_ld(src + (long)min(a0 + 4 * j, th + 1) * g.pitch);
    // The source (padded cell (sr, sc)) starts at +inf in D and takes its 0 here, inside its tile, so
    // that it counts as a cell that fell: on a tile edge or corner it marks the tiles it is the halo of.
    // (Written by the lane that stores that cell: a separate store raced with it -- r6u / r6v, an image
    // left at -1.)
    const bool s_here = sr > r0 && sr <= r0 + th && sc > c0 && sc <= c0 + tw;
    const int sa = s_here ? sr - r0 : -1, sb = sc - c0;
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (a0 + 4 * j <= th + 1 && lane <= tw + 1)
            L[(a0 + 4 * j) * GT_TP + lane] = (a0 + 4 * j == sa && lane == sb) ? 0.0f : old[j];
    grp.sync();
    // edge cells from the halo (read-only): top / bottom rows from rows 0 / th + 1, left / right columns
    // from columns 0 / tw + 1; straight weight 1, diagonals sqrt(2) (pyx:30-32); |-inf| = +inf passes nothing
    for (int k = t; k < 2 * tw + 2 * th; k += grp.n) {
        int a, b, ha, hb, da, db;  // the edge cell, its straight halo neighbour, the diagonal step along the edge
        if (k < 2 * tw) { b = 1 + k % tw; a = k < tw ? 1 : th; ha = k < tw ? 0 : th + 1; hb = b; da = 0; db = 1; }
        else { const int q = k - 2 * tw; a = 1 + q % th; b = q < th ? 1 : tw; hb = q < th ? 0 : tw + 1; ha = a; da = 1; db = 0; }
        const float s0 = fabsf(L[ha * GT_TP + hb]) + 1.0f;
        const float s1 = fabsf(L[(ha - da) * GT_TP + hb - db]) + SQRT2F;
        const float s2 = fabsf(L[(ha + da) * GT_TP + hb + db]) + SQRT2F;
        const float m = fminf(fminf(s0, s1), s2);
        if (m < L[a * GT_TP + b]) {  // (blocked cells hold -inf: never) its row and column are dirty
            lds_min(L + a * GT_TP + b, m);
            gt_mark_lines(sh.gdm[gi], a, b);
        }
    }
    if (t == 0 && sa > 0) gt_mark_lines(sh.gdm[gi], sa, sb);  // (the source's 0, set above)
    grp.sync();
    for (int round = 0;; round++) {
        uint64_t *dm = sh.gdm[gi];
        const bool c = dir == 0 ? gt_sweep<0>(L, th, tw, dm) : dir == 1 ? gt_sweep<1>(L, th, tw, dm)
                     : dir == 2 ? gt_sweep<2>(L, th, tw, dm) : gt_sweep<3>(L, th, tw, dm);
        if (c && (t & 63) == 0) __hip_atomic_store(&sh.chg[gi][round % 3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (t == 0) __hip_atomic_store(&sh.chg[gi][(round + 1) % 3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // (read 2 syncs ago)
        grp.sync();
        if (!gt_lds_ld(&sh.chg[gi][round % 3]) || gt_lds_ld(&sh.abort) || gt_lds_ld(&sh.bar[gi][2])) break;
        if (round > 4 * (GT_TT + 2) * (GT_TT + 2)) {  // (a bug guard: every round lowers a value)
            if (t == 0) __hip_atomic_store(&sh.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
        }
    }
    // write-back of the interior cells that fell (this group is the tile's only writer, so D still
    // holds what it loaded)
    unsigned em = 0;
    const int b = lane;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int a = a0 + 4 * j;
        if (a >= 1 && a <= th && b >= 1 && b <= tw) {
            const float v = L[a * GT_TP + b];
            if (v < old[j]) {
                D[(long)(r0 + a) * g.pitch + c0 + b] = v;  // (plain: see gl_tile_kernel's store rule)
                em |= (a == 1 ? 1u : 0u) | (a == th ? 2u : 0u) | (b == 1 ? 4u : 0u) | (b == tw ? 8u : 0u) |
                      (a == 1 && b == 1 ? 16u : 0u) | (a == 1 && b == tw ? 32u : 0u) | (a == th && b == 1 ? 64u : 0u) |
                      (a == th && b == tw ? 128u : 0u);
            }
        }
    }
    if (em) atomicOr(&sh.emask[gi], em);
    gl_drain();  // the stores are in L2 before any mark can send another group to read them
    grp.sync();
    return t == 0 ? gt_lds_ld(&sh.emask[gi]) : 0u;
}

// Batched GridGraph(grid).shortest_path_image(source) for windows of up to GT_MAXT tiles, one
// 1024-thread workgroup per query: same arguments, results and scratch layout as gl_sssp_kernel.
// Store rule: every store to D is a PLAIN store and every load of D an agent-scope (sc1, L1-bypassing)
// load.  The workgroup's waves share one CU, so one XCD's L2, where plain stores land: a store drained
// (vmcnt 0) before the mark that sends another group to the cells is seen by that group's loads, and
// the kernel's end writes the lines back for gl_path_kernel.
__global__ void __launch_bounds__(GT_NT) gl_tile_kernel(int H, int W, const uint8_t *__restrict__ grids, long grid_stride,
                                                       const int32_t *__restrict__ sources, int wi0, int wj0, int wh, int ww,
                                                       float *scratch, long scratch_stride, float *__restrict__ out,
                                                       unsigned *fault)
{
    __shared__ GtShared sh;
    __shared__ float tiles[GT_GROUPS * GT_BUF];
    const int b = blockIdx.x, tid = threadIdx.x;
    const uint8_t *grid = grids + b * grid_stride;
    const GlDims g = gl_dims(wh, ww);
    float *D = scratch + b * scratch_stride;
    const int si = sources[2 * b], sj = sources[2 * b + 1];
    const bool s_in = si >= wi0 && si < wi0 + wh && sj >= wj0 && sj < wj0 + ww && grid[(long)si * W + sj] != 0;
    const int ntj = (ww + GT_TT - 1) / GT_TT, nt = gt_tiles(wh, ww);
    if (nt > GT_MAXT) {  // (the host dispatches such windows to gl_sssp_kernel: a guard for the LDS tables)
        if (tid == 0) post_faults(fault, SIMAPS_FAULT_DESCRIPTOR);
        return;
    }
    // (rows by wave, columns by lane: no 64-bit index division; four independent loads in flight per
    // lane before their stores)
    for (int r = tid >> 6; r < wh + 2; r += GT_NT / 64) {
        const uint8_t *grow = grid + (long)(wi0 + r - 1) * W + wj0 - 1;
        float *drow = D + (long)r * g.pitch;
        const bool in_r = r >= 1 && r <= wh;
        for (int c0 = tid & 63; c0 < g.pitch; c0 += 256) {
            unsigned gb[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int c = c0 + 64 * q;
                gb[q] = (in_r && c >= 1 && c <= ww) ? grow[c] : 0u;
            }
#pragma unroll
            for (int q = 0; q < 4; q++)  // (the source too is +inf here: gt_process sets it)
                if (c0 + 64 * q < g.pitch) drow[c0 + 64 * q] = gb[q] ? INFINITY : -INFINITY;
        }
    }
    for (int k = tid; k < nt; k += GT_NT) sh.ring[k] = GT_EMPTY;
    for (int k = tid; k < (nt + 3) / 4; k += GT_NT) sh.st[k] = 0u;
    if (tid < GT_GROUPS * 4) (&sh.bar[0][0])[tid] = 0u;
    if (tid == 0) {
        sh.head = sh.tail = sh.outstanding = sh.processed = sh.abort = 0u;
        for (int q = 0; q < GT_GROUPS; q++) sh.emask[q] = 0u;
    }
    gl_drain();
    __syncthreads();
    if (tid == 0 && s_in) gt_mark(sh, ((si - wi0) / GT_TT) * ntj + (sj - wj0) / GT_TT, nt);
    __syncthreads();
    const int gi = tid >> 8;
    const Group grp{tid & 255, 256, sh.bar[gi], 4};
    lds_float *L = (lds_float *)(tiles + gi * GT_BUF + GT_PAD * GT_TP);  // (ds_* addressing)
    // processings: a bug guard.  Random grids take 2-3 per tile; a spiral corridor with 1-cell walls
    // crosses every tile ~31 times each way and takes ~60 (tools/tile_sssp_model.py), so 4x that.
    const unsigned cap = 256u * (unsigned)nt + 4096u;
    bool again = false;
    int cur = -1;
    for (;;) {
        if (grp.t == 0) {
            if (!again) cur = gt_pop(sh, nt);
            if (cur >= 0 && atomicAdd(&sh.processed, 1u) >= cap) {
                __hip_atomic_store(&sh.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                cur = -1;
            }
            sh.gtile[gi] = cur;
            sh.chg[gi][0] = sh.chg[gi][1] = sh.chg[gi][2] = 0u;
            sh.emask[gi] = 0u;
            sh.gdm[gi][0] = sh.gdm[gi][1] = sh.gdm[gi][2] = sh.gdm[gi][3] = 0ull;
        }
        grp.sync();
        const int tile = __builtin_amdgcn_readfirstlane(sh.gtile[gi]);  // (wave-uniform)
        if (tile < 0) break;
        if (gt_lds_ld(&sh.bar[gi][2])) {  // (a bug guard: a group barrier timed out -- stop the query)
            if (grp.t == 0) __hip_atomic_store(&sh.abort, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
        }
        const int ti = tile / ntj, tj = tile - ti * ntj;
        const unsigned em = gt_process(sh, L, D, g, ti, tj, grp, gi, si - wi0 + 1, sj - wj0 + 1);
        if (grp.t == 0) {
            const int nti = (wh + GT_TT - 1) / GT_TT;
            const bool up = ti > 0, dn = ti + 1 < nti, lf = tj > 0, rt = tj + 1 < ntj;
            if ((em & 1u) && up) gt_mark(sh, tile - ntj, nt);
            if ((em & 2u) && dn) gt_mark(sh, tile + ntj, nt);
            if ((em & 4u) && lf) gt_mark(sh, tile - 1, nt);
            if ((em & 8u) && rt) gt_mark(sh, tile + 1, nt);
            if ((em & 16u) && up && lf) gt_mark(sh, tile - ntj - 1, nt);
            if ((em & 32u) && up && rt) gt_mark(sh, tile - ntj + 1, nt);
            if ((em & 64u) && dn && lf) gt_mark(sh, tile + ntj - 1, nt);
            if ((em & 128u) && dn && rt) gt_mark(sh, tile + ntj + 1, nt);
            again = gt_finish(sh, tile);
        }
    }
    __syncthreads();
    if (tid == 0) {
        const unsigned ab = sh.abort;
        unsigned f = ab == 1u ? SIMAPS_FAULT_ROUNDS : ab ? SIMAPS_FAULT_TIMEOUT : 0u;
        for (int q = 0; q < GT_GROUPS; q++)
            if (sh.bar[q][2]) f |= SIMAPS_FAULT_TIMEOUT;
        post_faults(fault, f);
    }
    if (!out) return;
    for (int i = tid >> 6; i < H; i += GT_NT / 64) {
        float *orow = out + (long)b * H * W + (long)i * W;
        const int r = i - wi0;
        const bool rin = r >= 0 && r < wh;
        const float *drow = D + (long)(r + 1) * g.pitch + 1 - wj0;
        for (int j0 = tid & 63; j0 < W; j0 += 256) {
            float d[4];  // (four independent loads in flight per lane before their stores)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = j0 + 64 * q, c = j - wj0;
                d[q] = (rin && j < W && c >= 0 && c < ww) ? gl_ld(drow + j) : -INFINITY;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = j0 + 64 * q;
                if (j < W) {
                    float v = (i == si && j == sj) ? 0.0f : -1.0f;
                    if (d[q] >= 0.0f && d[q] != INFINITY) v = d[q];
                    orow[j] = v;
                }
            }
        }
    }
}

// Per-query scratch of gl_path_kernel, in int32 / float32 units of `cells` (padded cells) and `n`
// (window cells + 1): fix [cells] (gl_sssp_kernel's fixpoint), dist [cells], pin [cells], queue [n]
// (ring: live entries <= free cells), dense [n], chain [n], stack [2 n].
__host__ __device__ inline long gl_path_words(int wh, int ww)
{
    const long cells = (long)(wh + 2) * (ww + 2), n = (long)wh * ww + 1;
    return 3 * cells + 5 * n;
}

// pyx:30 directions: 1 + k in pin bits 0-3; the edge's cell offset in the padded layout
__device__ __forceinline__ long gl_dir_off(int k, int pitch)
{
    const int di = k < 2 ? 0 : (k < 5 ? -1 : 1);
    const int dj = k < 2 ? (k == 0 ? -1 : 1) : ((k - 2) % 3) - 1;
    return (long)di * pitch + dj;
}

// GridGraph(grid).shortest_path(source, target) (pyx:121-154) on windows of any size, one wave per
// query, after gl_sssp_kernel left the fixpoint from the same source in `fix`.  Output as
// grid_path_kernel: waypoint cells source first, count or -needed.
__global__ void __launch_bounds__(64) gl_path_kernel(int H, int W, const uint8_t *__restrict__ grids, long grid_stride,
                                                    const int32_t *__restrict__ sources, const int32_t *__restrict__ targets,
                                                    int wi0, int wj0, int wh, int ww, int *scratch, long scratch_stride,
                                                    int max_pts, int32_t *__restrict__ out_ij, int32_t *__restrict__ out_n,
                                                    unsigned *fault)
{
    const int b = blockIdx.x, lane = threadIdx.x;
    const uint8_t *grid = grids + b * grid_stride;
    const GlDims g = gl_dims(wh, ww);
    const int P = g.pitch;
    const long n1 = (long)wh * ww + 1;
    int *base = scratch + b * scratch_stride;
    const float *fix = reinterpret_cast<const float *>(base);
    float *dist = reinterpret_cast<float *>(base + g.cells);
    int *pin = base + 2 * g.cells;
    int *queue = base + 3 * g.cells;
    int *dense = queue + n1;
    int *chain = dense + n1;
    int *stack = chain + n1;
    const int si = sources[2 * b], sj = sources[2 * b + 1], ti = targets[2 * b], tj = targets[2 * b + 1];
    int32_t *o = out_ij + (long)b * max_pts * 2;
    const bool s_in = si >= wi0 && si < wi0 + wh && sj >= wj0 && sj < wj0 + ww;
    const bool t_in = ti >= wi0 && ti < wi0 + wh && tj >= wj0 && tj < wj0 + ww;
    // a source outside the window or blocked has no edges (pyx:56) and a target outside the window is
    // never reached: the parent walk stops at once and the path is [target]
    if (!(s_in && t_in && grid[(long)si * W + sj] != 0)) {
        if (lane == 0) { o[0] = ti; o[1] = tj; out_n[b] = 1; }
        return;
    }
    const long su = (long)(si - wi0 + 1) * P + (sj - wj0 + 1), tv = (long)(ti - wi0 + 1) * P + (tj - wj0 + 1);
    // (1) SPFA arrays: distances +inf on free cells (the reference's 2 * V: no path reaches it), -inf
    // on blocked and border cells (never relaxed), pin 0; the queue holds the source (pyx:79-88).
    // This wave is the only user of its arrays, so they are read through the L1 (plain loads); every
    // pop's stores are drained (gl_drain) before the next pop's loads issue.
    for (long k = lane; k < g.cells; k += 64) {
        const float fv = fix[k];
        dist[k] = k == su ? 0.0f : (fv == -INFINITY ? -INFINITY : INFINITY);
        pin[k] = k == su ? GL_INQ : 0;
    }
    if (lane == 0) queue[0] = (int)su;
    gl_drain();
    unsigned fault_bits = 0;
    const float finT = fix[tv];  // the target's fixpoint distance
    // The pop cap (a bug guard: a correct SPFA never reaches it) scales with the window: the
    // reference's linear queue holds 8 V entries (pyx:78), so its SPFA never pops more than that.
    const long pop_cap = SIMAPS_POP_CAP > 8L * wh * ww + 1 ? (long)SIMAPS_POP_CAP : 8L * wh * ww + 1;
    const int k8 = lane < 8 ? lane : 8;
    const int off = lane < 8 ? (int)gl_dir_off(lane, P) : 0;  // lane 8: the popped vertex itself
    const float wl = (lane >= 2 && lane < 8 && lane != 3 && lane != 6) ? SQRT2F : 1.0f;
    // the queue: live slots qh .. qt (mod QR), cnt entries; its front u and (cnt >= 2) second s2 are
    // kept in registers, so a pop's reads -- u's edge heads, the entry after s2, s2's distance -- go
    // out together in one round
    // (cell and slot indices in 32 bits: a window has < 2^31 padded cells, H, W <= 32767; 64-bit index
    // arithmetic was a good part of each pop's serial instruction stream)
    const int QR = (int)n1;
    int qh = 0, qt = 0, cnt = 1, u = (int)su, s2 = -1;
    long pops = 0, lim = GL_CHECK;
    // Early exit, incremental (round 6): the chain from the target up to (not including) wchk holds its
    // fixpoint distances, so its parents can no longer change (pyx:97-99 sets a parent only on a strict
    // improvement) and each check resumes at wchk instead of walking the chain again.  (Round 5
    // re-walked it at doubling intervals, 64, 128, ... pops, and so stopped up to twice as late:
    // modelled on 500^2 grids, the chain was final after 54-91 % of the pops the old schedule ran.)
    int wchk = (int)tv;
    long chk_steps = 0;
    bool early = false;
    // an unreachable (+inf) or blocked (-inf) target never gets a parent (pin[tv] stays 0 unless it is
    // the source): the path is [target] whatever the SPFA does, so it is not run
    if (!(finT > -INFINITY && finT < INFINITY)) cnt = 0;
#ifdef SIMAPS_GL_STATS
    const long t_start = __builtin_readcyclecounter();
#endif
    while (cnt > 0) {
        // (2) pop u; its edges in pyx order on lanes 0-7 (pyx:89-101), lane 8 u itself
        const int q2 = qh + 1 == QR ? 0 : qh + 1, q3 = q2 + 1 == QR ? 0 : q2 + 1;
        const int v = u + off;
        const float dv = lane <= 8 ? dist[v] : 0.0f;
        const int pv = lane <= 8 ? pin[v] : 0;
        const int third_l = (lane == 9 && cnt >= 3) ? queue[q3] : -1;
        const float dfr_l = (lane == 10 && cnt >= 2) ? dist[s2] : 0.0f;
        const int fr = cnt >= 2 ? s2 : -1;  // the front after this pop (queue[head + 1])
        // (lane values to the wave by v_readlane, uniform lane index: a ds_bpermute (__shfl) is an LDS
        // round trip on the pop's serial chain, several per pop)
        const int third = gl_lane(third_l, 9);
        const float dfr = gl_lane(dfr_l, 10);  // its distance before this pop
        qh = q2;
        cnt--;
        const float du = gl_lane(dv, 8);
        const float nd = du + wl;
        const bool imp = lane < 8 && nd < dv;
        if (imp) {
            dist[v] = nd;
            pin[v] = GL_INQ | (k8 + 1);
        }
        if (lane == 8) pin[u] = pv & 15;  // in_queue[u] = 0 (pyx:92)
        // (3) pushes in edge order with the SLF swap against the front (pyx:102-107); the front's
        // distance as of each edge: lowered by this pop's own edge to it, if any.  Queued heads are
        // never pushed (the original front too, also after a swap moved it to the tail).
        uint64_t todo = __ballot(imp && ((pv & GL_INQ) == 0 || v == fr));
        int f = fr, nsec = cnt >= 2 ? third : -1;
        const int q2n = qh + 1 == QR ? 0 : qh + 1;  // the slot after the front
        float df = dfr;
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int vk = gl_lane(v, k);
            const float ndk = gl_lane(nd, k);
            if (gl_lane(pv, k) & GL_INQ) {  // the front itself improved (queued: no push)
                if (vk == f) df = ndk;
                continue;
            }
            qt = qt + 1 == QR ? 0 : qt + 1;
            cnt++;
            int content = vk;
            if (cnt == 1) {  // (the queue was empty: tail == head + 1 == this slot)
                f = vk;
                df = ndk;
            } else if (ndk < df) {
                if (lane == 0) queue[qh] = (int)vk;
                content = f;
                f = vk;
                df = ndk;
            }
            if (lane == 0) queue[qt] = (int)content;
            if (qt == q2n) nsec = content;
        }
        u = f;
        s2 = nsec;
        gl_drain();  // (a timing variant without this wait was only 4 % faster: profiles/r5h_*)
        if (++pops < lim) continue;
        if (pops >= pop_cap) {
            if (cnt > 0) fault_bits |= SIMAPS_FAULT_ROUNDS;  // the cap stopped a live queue
            break;
        }
        // (4) early exit: the target at its fixpoint distance and then every vertex of its chain
        while (wchk != su && chk_steps <= n1) {  // (the step bound guards a parent cycle: never)
            if (dist[wchk] != (wchk == tv ? finT : fix[wchk])) break;  // not final yet: resume here
            const int p = pin[wchk] & 15;
            if (!p) break;
            wchk -= gl_dir_off(p - 1, P);
            chk_steps++;
        }
        if (wchk == su) { early = true; break; }
        lim = pops + GL_CHECK < pop_cap ? pops + GL_CHECK : pop_cap;
    }
#ifdef SIMAPS_GL_STATS  // (diagnostic build: tools/debug/gl_pipe_stats.py)
    if (lane == 0) printf("glser pops %ld cycles %ld\n", pops, (long)__builtin_readcyclecounter() - t_start);
#endif
    (void)early;
    // (5) dense path: parents from the target back to the source (pyx:131-138)
    int nd = 0;
    if (lane == 0) {
        long w = tv;
        dense[nd++] = (int)w;
        while (w != su) {
            const int p = gl_ldi(pin + w) & 15;
            if (!p) break;
            w -= gl_dir_off(p - 1, P);
            dense[nd++] = (int)w;
        }
    }
    nd = __shfl(nd, 0);
    gl_drain();
    auto rc_of = [&](int q, int &r, int &c) { r = q / P - 1 + wi0; c = q % P - 1 + wj0; };
    // (6) approximate_polygon(dense, tolerance=1) (skimage 0.18.3 measure/_polygon.py), as path_core
    for (int k = lane; k < nd; k += 64) chain[k] = (k == 0 || k == nd - 1) ? 1 : 0;
    gl_drain();
    {
        long sp = 1, iters = 0;
        if (lane == 0) { stack[0] = 0; stack[1] = nd - 1; }
        gl_drain();
        while (sp > 0 && ++iters <= 2L * nd) {
            sp--;
            const int start = gl_ldi(stack + 2 * sp), end = gl_ldi(stack + 2 * sp + 1);
            int r0, c0, r1, c1;
            rc_of(gl_ldi(dense + start), r0, c0);
            rc_of(gl_ldi(dense + end), r1, c1);
            const long dr = r1 - r0, dc = c1 - c0;
            const double ang = -atan2((double)dr, (double)dc);
            const double sn = sin(ang), cs = cos(ang);
            const double sdist = (double)c0 * sn + (double)r0 * cs;
            double best = -1.0;
            int besti = -1;
            for (int k = start + 1 + lane; k < end; k += 64) {
                int rr, cc;
                rc_of(gl_ldi(dense + k), rr, cc);
                const long dr0 = rr - r0, dc0 = cc - c0, dr1 = rr - r1, dc1 = cc - c1;
                const bool perp = dr0 * dr + dc0 * dc > 0 && -dr1 * dr - dc1 * dc > 0;
                double d;
                if (perp) d = fabs(((double)rr * cs + (double)cc * sn) - sdist);
                else d = fmin(sqrt((double)(dc0 * dc0 + dr0 * dr0)), sqrt((double)(dc1 * dc1 + dr1 * dr1)));
                if (d > best) { best = d; besti = k; }
            }
            for (int o2 = 32; o2 > 0; o2 >>= 1) {  // wave argmax, first index on ties (np.argmax)
                const double ob = __shfl_xor(best, o2);
                const int oi = __shfl_xor(besti, o2);
                if (ob > best || (ob == best && oi >= 0 && (besti < 0 || oi < besti))) { best = ob; besti = oi; }
            }
            if (best > 1.0) {
                if (lane == 0) {
                    gl_sti(stack + 2 * sp, besti);
                    gl_sti(stack + 2 * sp + 1, end);
                    gl_sti(stack + 2 * sp + 2, start);
                    gl_sti(stack + 2 * sp + 3, besti);
                    gl_sti(chain + besti, 1);
                }
                sp += 2;
            }
            gl_drain();
        }
    }
    // (7) sparse points (chain-flagged, in order) into `stack`, then the line-of-sight pruning on the
    // grid (pyx:143-150: a line is blocked by any cell != 1) and the reversal (pyx:152)
    int *sparse = stack;
    int m = 0;
    for (int k0 = 0; k0 < nd; k0 += 64) {
        const int k = k0 + lane;
        const bool fl = k < nd && gl_ldi(chain + k);
        const uint64_t bm = __ballot(fl);
        if (fl) gl_sti(sparse + m + __popcll(bm & ((1ull << lane) - 1)), gl_ldi(dense + k));
        m += __popcll(bm);
    }
    gl_drain();
    int *kept = chain;  // (chain flags are no longer read)
    int cnt_out = 0;
    if (m > 0) {
        if (lane == 0) gl_sti(kept, gl_ldi(sparse));
        cnt_out = 1;
        for (int k = 1; k < m - 1; k++) {
            gl_drain();
            int ra, ca, rb, cb;
            rc_of(gl_ldi(kept + cnt_out - 1), ra, ca);
            rc_of(gl_ldi(sparse + k + 1), rb, cb);
            const int len = max(abs(rb - ra), abs(cb - ca)) + 1;
            bool blocked = false;
            for (int t = lane; t < len; t += 64) {
                int pr, pc;
                line_pixel(ra, ca, rb, cb, t, pr, pc);
                blocked |= grid[(long)pr * W + pc] != 1;
            }
            if (__ballot(blocked) != 0) {
                if (lane == 0) gl_sti(kept + cnt_out, gl_ldi(sparse + k));
                cnt_out++;
            }
        }
        if (m > 1) {
            if (lane == 0) gl_sti(kept + cnt_out, gl_ldi(sparse + m - 1));
            cnt_out++;
        }
    }
    gl_drain();
    if (cnt_out > max_pts) {
        if (lane == 0) out_n[b] = -cnt_out;
    } else {
        for (int k = lane; k < cnt_out; k += 64) {
            int r, c;
            rc_of(gl_ldi(kept + cnt_out - 1 - k), r, c);
            o[2 * k] = r;
            o[2 * k + 1] = c;
        }
        if (lane == 0) out_n[b] = cnt_out;
    }
    if (lane == 0) post_faults(fault, fault_bits);
}
