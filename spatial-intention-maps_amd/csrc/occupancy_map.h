// OccupancyMap (envs.py:2409-2524) as its own drop-in, round 6: the maps OccupancyMap.update derives
// from the occupancy grid, and its EDT snap, as outputs of the C ABI (simaps_occupancy_scatter /
// simaps_build_cspace / simaps_snap_sources, include/simaps.h).  Inside the get_state / path kernels
// these maps never leave the CU; here they are written out for a caller of OccupancyMap itself.
// Included by simaps.hip inside its device namespace (after the ingest kernels, whose pixel clip it
// shares).
//
//   occupancy_scatter_kernel  OccupancyMap.update's obstacle scatter (envs.py:2445-2450): every point
//                             whose segmentation value np.isclose()s the obstacle value marks its
//                             Mapper.position_to_pixel_indices pixel (envs.py:2391-2397) occupied.
//   occupancy_map_kernel      per agent, the cspace of build_cspace (envs.py:2453: 1 - max(1 - room_mask,
//                             binary_dilation(occupancy, disk(floor(RADIUS * 96))))), written over the
//                             whole grid; cspace_thin (2456: 1 - binary_dilation(min(room_mask,
//                             occupancy), disk(3))); and closest_cspace_indices (2455: scipy's EDT
//                             feature transform of 1 - cspace) at query pixels.  grid.y = agent,
//                             grid.x = a slice of OCC_SNAP_PER_WG query pixels; every workgroup builds
//                             the agent's cspace in LDS (~3 us), workgroup 0 also writes the images.

constexpr int OCC_SNAP_PER_WG = 64;  // query pixels per workgroup: 16 per wave, one wave per query

struct OccHdr {  // the rect fields thin_free reads
    int h, w, i0, j0;
};

__global__ void __launch_bounds__(256) occupancy_scatter_kernel(int H, int W, int P, const simaps_agent *__restrict__ agents,
                                                               const float *__restrict__ points,
                                                               const float *__restrict__ seg, double value,
                                                               uint8_t *__restrict__ occupancy)
{
    const int n = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= P) return;
    const size_t q = (size_t)n * P + k;
    // np.isclose(seg, value): |seg - value| <= 1e-8 + 1e-5 |value|, in float64 (numpy promotes the
    // float32 array against the Python float); NaN is never close
    const double s = (double)seg[q];
    if (!(fabs(s - value) <= 1e-8 + 1e-5 * fabs(value))) return;
    // Mapper.position_to_pixel_indices on float32 points: floor(H / 2 - y * 96), floor(W / 2 + x * 96)
    // in float32, astype(int32), clipped (the ingest kernel's rule)
    const float h2 = (float)((double)H / 2), w2 = (float)((double)W / 2);
    const float x = points[3 * q], y = points[3 * q + 1];
    const int pi = ingest_clip(floorf(h2 - y * 96.0f), H), pj = ingest_clip(floorf(w2 + x * 96.0f), W);
    occupancy[(size_t)agents[n].map_slot * H * W + (size_t)pi * W + pj] = 1;
}

__global__ void __launch_bounds__(PNT) occupancy_map_kernel(simaps_config cfg, Geometry geo,
                                                            const simaps_agent *__restrict__ agents,
                                                            const simaps_env *__restrict__ envs,
                                                            const simaps_robot *__restrict__ robots,
                                                            const uint8_t *__restrict__ occupancy, uint8_t *cspace,
                                                            uint8_t *thin, const int32_t *__restrict__ pixels, int Q,
                                                            int32_t *snapped, unsigned *fault)
{
    __shared__ __attribute__((aligned(16))) SsspScratch S;
    __shared__ int rad, bad;
    const int n = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = cfg.H, W = cfg.W;
    const OccHdr hd{cfg.room_h, cfg.room_w, cfg.room_i0, cfg.room_j0};
    const simaps_agent ag = agents[n];
    if (tid == 0) {
        bool b;
        rad = geo.cspace_r[agent_robot_type(ag, envs, robots, b)];  // floor(RADIUS * 96) of its class
        bad = b;
    }
    lds_barrier();
    const Group g{tid, PNT, nullptr, PNT / 64};
    build_cspace<PNT>(S, nullptr, hd.h, hd.w, rad, g, nullptr, 0, nullptr, occupancy + (size_t)ag.map_slot * H * W, H,
                      W, hd.i0, hd.j0);  // (ends with a sync: S.freeb and S.win are complete)
    if (chunk == 0) {
        if (tid == 0 && bad) post_faults(fault, SIMAPS_FAULT_DESCRIPTOR);
        const size_t base = (size_t)n * H * W;
        for (int i = wave; i < H; i += PNT / 64) {  // a wave per row, a lane per column
            const int r = i - hd.i0;
            const bool row_in = r >= 0 && r < hd.h;
            const bool near = i >= hd.i0 - 3 && i < hd.i0 + hd.h + 3;  // disk(3) reach of the rect
            for (int j = lane; j < W; j += 64) {
                const int c = j - hd.j0;
                if (cspace) cspace[base + (size_t)i * W + j] = row_in && c >= 0 && c < hd.w && b_test(S.freeb[r], c) ? 1 : 0;
                if (thin)  // no in-room obstacle within disk(3): 1 (all pixels farther than 3 from the rect)
                    thin[base + (size_t)i * W + j] = near && j >= hd.j0 - 3 && j < hd.j0 + hd.w + 3 ? (thin_free(hd, S, i, j) ? 1 : 0) : 1;
            }
        }
    }
    if (!snapped) return;
    const int q1 = min(Q, (chunk + 1) * OCC_SNAP_PER_WG);
    for (int q = chunk * OCC_SNAP_PER_WG + wave; q < q1; q += PNT / 64) {
        const size_t o = ((size_t)n * Q + q) * 2;
        const int qi = __builtin_amdgcn_readfirstlane(pixels[o]), qj = __builtin_amdgcn_readfirstlane(pixels[o + 1]);
        int si = -1, sj = -1;
        if (qi >= 0 && qi < H && qj >= 0 && qj < W) {
            const int r = qi - hd.i0, c = qj - hd.j0;
            if (r >= 0 && r < hd.h && c >= 0 && c < hd.w && b_test(S.freeb[r], c)) {
                si = qi;  // a free pixel is its own nearest free cell (EDT distance 0)
                sj = qj;
            } else {
                snap_wave(S.freeb, hd.h, hd.w, hd.i0, hd.j0, qi, qj, [&](int a, int b) { si = a; sj = b; });
            }
        }
        if (lane == 0) {
            snapped[o] = si;
            snapped[o + 1] = sj;
        }
    }
}
