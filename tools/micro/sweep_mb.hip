// Sweep-step microbenchmark (diagnostic, not part of the product): the SSSP line step of
// simaps.hip (sweep_asm, CPL 2: two cells per lane) run by NW waves of one 1024-thread workgroup,
// each on its own LDS array, so that the per-step cost can be split between VALU issue, the LDS
// prefetch reads and the LDS atomic mins, with 1 .. 8 concurrent sweep waves (wave w -> SIMD w % 4).
// Build variants with -DMB_NOMIN (no ds_min), -DMB_NOREAD (no reads), -DMB_WIDE (the lane's two
// cells 64 apart instead of adjacent: conflict-free LDS accesses).
//   hipcc -O3 --offload-arch=gfx950 [-D...] tools/micro/sweep_mb.hip -o /tmp/sweep_mb && /tmp/sweep_mb
#include <hip/hip_runtime.h>
#include <cstdio>

#ifdef MB_NOMIN
#define MB_MIN(x) ""
#else
#define MB_MIN(x) x
#endif
#ifdef MB_NOREAD
#define MB_RD(x) ""
#define MB_WAIT "s_waitcnt lgkmcnt(0)\n\t"
#elif defined(MB_NOMIN)
#define MB_RD(x) x
#define MB_WAIT "s_waitcnt lgkmcnt(2)\n\t"
#else
#define MB_RD(x) x
#define MB_WAIT "s_waitcnt lgkmcnt(6)\n\t"
#endif
#ifdef MB_WIDE
#define MB_SA "256"
#else
#define MB_SA "4"
#endif

__global__ void __launch_bounds__(1024) sweep_mb(unsigned long long *out, int steps, int nwaves, int pitch)
{
    __shared__ float lds[36 * 1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < 36 * 1024; k += 1024) lds[k] = 1e30f;
    __syncthreads();
    if (wave >= nwaves) return;
#ifdef MB_WIDE
    const int cell = lane;
#else
    const int cell = 2 * lane;
#endif
    float *base = lds + wave * 2200 + cell;
    unsigned va = (unsigned)(uintptr_t)base;
    float p0 = 1.0f, p1 = 2.0f, one = 1.0f, s2 = 1.41421354f, X = 1e30f, acc = 0.0f;
    float a, b, c, d, e, f, r0 = 0.0f, r1 = 0.0f, q0 = 0.0f, q1 = 0.0f;
    const unsigned stride = (unsigned)pitch * 4;
    const int n = steps / 2;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int t = 0; t < n; t++) {
        // two steps per iteration (prefetch ring of 2 lines), line offsets wrap inside the wave's array
        asm volatile(
#define STEP(R0, R1)                                                                                  \
            "v_add_f32_e64 %[a], |%[p0]|, %[one]\n\t"                                                 \
            "v_add_f32_e64 %[d], |%[p1]|, %[one]\n\t"                                                 \
            "v_add_f32_e64 %[c], |%[p1]|, %[s2]\n\t"                                                  \
            "v_add_f32_e64 %[e], |%[p0]|, %[s2]\n\t"                                                  \
            "v_add_f32_dpp %[b], |%[p1]|, %[s2] wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
            "v_add_f32_dpp %[f], |%[p0]|, %[s2] wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
            "v_min3_f32 %[a], %[a], %[b], %[c]\n\t"                                                   \
            "v_min3_f32 %[d], %[d], %[e], %[f]\n\t"                                                   \
            MB_MIN("ds_min_f32 %[va], %[a]\n\t")                                                      \
            MB_MIN("ds_min_f32 %[va], %[d] offset:" MB_SA "\n\t")                                     \
            MB_WAIT                                                                                   \
            "v_minimum3_f32 %[p0], %[a], %[" #R0 "], %[X]\n\t"                                        \
            "v_minimum3_f32 %[p1], %[d], %[" #R1 "], %[X]\n\t"                                        \
            "v_sub_f32 %[b], %[a], %[" #R0 "]\n\t"                                                    \
            "v_sub_f32 %[e], %[d], %[" #R1 "]\n\t"                                                    \
            MB_RD("ds_read_b32 %[" #R0 "], %[va] offset:2048\n\t")                                    \
            MB_RD("ds_read_b32 %[" #R1 "], %[va] offset:(2048+" MB_SA ")\n\t")                        \
            "v_min3_f32 %[acc], %[acc], %[b], %[e]\n\t"                                               \
            "v_xor_b32 %[va], %[va], %[st]\n\t"
            STEP(r0, r1) STEP(q0, q1)
#undef STEP
            : [p0] "+v"(p0), [p1] "+v"(p1), [acc] "+v"(acc), [va] "+v"(va), [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c),
              [d] "=&v"(d), [e] "=&v"(e), [f] "=&v"(f), [r0] "+v"(r0), [r1] "+v"(r1), [q0] "+v"(q0), [q1] "+v"(q1)
            : [one] "v"(one), [s2] "v"(s2), [X] "v"(X), [st] "v"(stride)
            : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[wave] = t1 - t0;
    if (acc == 12345.0f) lds[0] = p0 + p1;
}

int main()
{
    unsigned long long *d, h[16];
    hipMalloc(&d, 16 * sizeof(unsigned long long));
    const int steps = 4000;
    for (int nw : {1, 2, 4, 8, 16}) {
        for (int rep = 0; rep < 2; rep++)
            hipLaunchKernelGGL(sweep_mb, dim3(1), dim3(1024), 0, 0, d, steps, nw, 95);
        hipDeviceSynchronize();
        hipMemcpy(h, d, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double mx = 0;
        for (int w = 0; w < nw; w++) mx = mx > h[w] ? mx : (double)h[w];
        printf("waves=%2d  %.1f cycles/step (slowest wave)\n", nw, mx / steps);
    }
    return 0;
}
