// The global maps of Mapper.get_state(save_figures=True) (envs.py:2115-2182) as outputs, round 6: the
// fused kernel only ever builds the 136 x 136 crop of each map around its agent; the reference's debug
// path saves the whole-room maps too.  One workgroup per agent writes, over the whole [H, W] grid:
//   overhead   Mapper._create_global_overhead_map (2244-2249): the overhead map without robots, every
//              robot's rotated mask stamped in with its group's seg value;
//   robot      Mapper._create_global_robot_map(seg=False) (2251-2276): 1 (0.5 for a lifting robot not
//              lifting, the lifted-cube mask while lifting), max over robots;
//   history /  Mapper._create_global_intention_or_history_map (2302-2347) with encoding 'history' /
//   intention  the configuration's encoding: the other non-idle robots' paths, Bresenham lines with the
//              fp64 linspace ramp, max-combined, grey-dilated by the cross for thickness 2.
// The same device code as the fused kernel's stamps and raster phases (robot_params, rot_src, the mask
// windows, seg_table and its pixel / value rules), on global coordinates.  Not a hot path: a debug
// export, any output may be NULL.  Included by simaps.hip inside its device namespace.

__global__ void __launch_bounds__(NT) global_maps_kernel(simaps_config cfg, Geometry geo,
                                                         const simaps_agent *__restrict__ agents,
                                                         const simaps_env *__restrict__ envs,
                                                         const simaps_robot *__restrict__ robots,
                                                         const double *__restrict__ paths,
                                                         const float *__restrict__ overhead, float *overhead_map,
                                                         float *robot_map, float *history_map, float *intention_map,
                                                         unsigned *fault)
{
    __shared__ __attribute__((aligned(16))) Shared sh;
    const int n = blockIdx.x, tid = threadIdx.x;
    const int H = cfg.H, W = cfg.W;
    const size_t base = (size_t)n * H * W;
    simaps_agent ag = agents[n];
    simaps_env ev = envs[ag.env];
    // descriptors come through the C ABI unchecked: clamp what would index past the LDS tables
    const bool bad = (unsigned)(ev.num_robots - 1) >= (unsigned)SIMAPS_MAX_ROBOTS || (unsigned)ag.robot >= (unsigned)ev.num_robots;
    ev.num_robots = min(max(ev.num_robots, 1), SIMAPS_MAX_ROBOTS);
    if ((unsigned)ag.robot >= (unsigned)ev.num_robots) ag.robot = 0;
    const simaps_robot *rb = robots + ev.robot_off;
    const int nr = ev.num_robots;
    if (tid == 0) {
        sh.nr = nr;
        sh.me = ag.robot;
        if (bad) post_faults(fault, SIMAPS_FAULT_DESCRIPTOR);
    }
    if (tid < nr) robot_params(sh.rob[tid], rb[tid], cfg, geo, H, W);
    if (tid >= 128 && tid < 128 + 5 * 24) sh.mwin[tid - 128] = geo.mbits[(tid - 128) / 24][(tid - 128) % 24];
    if (tid >= 256 && tid < 256 + 20) {
        const int q = tid - 256, m = q >> 2, f = q & 3;
        sh.mwin[120 + q] = f == 0 ? geo.mrow0[m] : f == 1 ? geo.mcol0[m] : f == 2 ? geo.mnrows[m] : geo.mncols[m];
    }
    __syncthreads();
    // ---- overhead / robot maps: per pixel, the robot-code bits of every robot whose box holds it (the
    // stamps phase's rule: rot_src into the class mask window, the lifted-cube window while lifting)
    if (overhead_map || robot_map) {
        for (int p = tid; p < H * W; p += NT) {
            const int gi = p / W, gj = p - (p / W) * W;
            unsigned code = 0;
            for (int k = 0; k < nr; k++) {
                const RobotP &P = sh.rob[k];
                if (gi < P.bi0 || gi > P.bi1 || gj < P.bj0 || gj > P.bj1) continue;
                const Rot R{P.c, P.s, P.f0, P.f1, P.S0, P.S1};
                int m0, m1;
                if (!rot_src(R, LW, gi - P.st_i, gj - P.st_j, m0, m1)) continue;
                const int *mt = reinterpret_cast<const int *>(sh.mwin + 120 + 4 * P.type);
                const int *mc = reinterpret_cast<const int *>(sh.mwin + 120 + 4 * 4);
                const int r = m0 - mt[0], cc = m1 - mt[1];
                if ((unsigned)r < (unsigned)mt[2] && (unsigned)cc < (unsigned)mt[3] && ((sh.mwin[P.type * 24 + r] >> cc) & 1u))
                    code |= P.code0;
                const int r2 = m0 - mc[0], c2 = m1 - mc[1];
                if (P.type == SIMAPS_LIFTING && P.lifting && (unsigned)r2 < (unsigned)mc[2] && (unsigned)c2 < (unsigned)mc[3] &&
                    ((sh.mwin[4 * 24 + r2] >> c2) & 1u))
                    code |= 1u << 5;
            }
            // bit g: seg value (g + 5) / 8 (robot_group_{g+1}); bit 4: 0.5; bit 5: 1.0 -- the max is the top bit
            const unsigned ms = code & 0xfu, mr = code >> 4;
            const float vseg = ms ? (float)(31 - __builtin_clz(ms) + 5) * 0.125f : 0.0f;
            if (overhead_map) overhead_map[base + p] = vseg > 0.0f ? vseg : overhead[(size_t)ag.map_slot * H * W + p];
            if (robot_map) robot_map[base + p] = (mr & 2u) ? 1.0f : ((mr & 1u) ? 0.5f : 0.0f);
        }
    }
    // ---- history / intention rasters over the whole grid (raster_lines' pixel and value rules, no tile)
    const float scale_f = (float)cfg.intention_map_scale;
    const int thick = cfg.intention_map_line_thickness;
    for (int pass = 0; pass < 2; pass++) {
        float *out = pass == 0 ? history_map : intention_map;
        if (!out) continue;
        const int enc = pass == 0 ? 4 : cfg.intention_map_encoding;
        unsigned *ou = reinterpret_cast<unsigned *>(out + base);
        for (int p = tid; p < H * W; p += NT) ou[p] = 0u;
        if (tid < nr) seg_table(sh, cfg, rb, paths, enc, tid, sh.me);
        // the zeros must be in L2 before any wave's atomicMax on them: a workgroup-scope barrier waits
        // for LDS only (s_waitcnt lgkmcnt), so an agent-scope fence drains this wave's stores first
        __threadfence();
        __syncthreads();  // (the zeros; the segment table)
        auto put = [&](int a, int b, float v) {  // max into (a, b) and, thick, its cross (grey dilation, disk(1))
            const unsigned u = __float_as_uint(v);  // v > 0: the uint order is the float order
            if ((unsigned)a < (unsigned)H && (unsigned)b < (unsigned)W) atomicMax(&ou[a * W + b], u);
            if (thick > 1) {
                if ((unsigned)(a - 1) < (unsigned)H && (unsigned)b < (unsigned)W) atomicMax(&ou[(a - 1) * W + b], u);
                if ((unsigned)(a + 1) < (unsigned)H && (unsigned)b < (unsigned)W) atomicMax(&ou[(a + 1) * W + b], u);
                if ((unsigned)a < (unsigned)H && (unsigned)(b - 1) < (unsigned)W) atomicMax(&ou[a * W + b - 1], u);
                if ((unsigned)a < (unsigned)H && (unsigned)(b + 1) < (unsigned)W) atomicMax(&ou[a * W + b + 1], u);
            }
        };
        if (enc == SIMAPS_ENC_CIRCLE) {
            if (tid < nr && tid != sh.me && !sh.rob[tid].idle && scale_f > 0.0f) put(sh.rob[tid].tpi, sh.rob[tid].tpj, scale_f);
        } else {
            for (int q = 0; q < nr * SEG_PER_ROBOT; q++) {
                if (q % SEG_PER_ROBOT >= sh.seg_robot_cnt[q / SEG_PER_ROBOT]) continue;
                const Seg &G = sh.seg[q];
                const int npix = G.last ? G.n : G.n - 1;  // non-final segments drop their last pixel
                const bool steep = G.dr > G.dc;
                const int major = steep ? G.dr : G.dc, minor = steep ? G.dc : G.dr;
                const int smaj = steep ? (G.ti - G.si > 0 ? 1 : -1) : (G.tj - G.sj > 0 ? 1 : -1);
                const int smin = steep ? (G.tj - G.sj > 0 ? 1 : -1) : (G.ti - G.si > 0 ? 1 : -1);
                for (int t = tid; t < npix; t += NT) {
                    int pr, pc;
                    if (t == G.n - 1) {  // skimage: rr[dc] = r1, cc[dc] = c1
                        pr = G.ti;
                        pc = G.tj;
                    } else {
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
                    if (v > 0.0f) put(pr, pc, v);
                }
            }
        }
        __syncthreads();  // (the next pass rewrites the segment table)
    }
}
