// Instruction issue / latency microbenchmark (diagnostic, not part of the product): one workgroup of
// NW waves on one CU; wave 0 times a loop of a given instruction pattern with s_memtime; the other
// waves (if any) spin on the same pattern so the SIMDs are shared like in the sweep phase.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP16(x) REP8(x) REP8(x)

template <int K>
__global__ void bench(unsigned long long *out, int iters, int active_waves, int active_lanes)
{
    const int wave = threadIdx.x >> 6;
    float a = threadIdx.x * 0.5f, b = 1.0f, c = 2.0f, d = 3.0f, e = 4.0f, f = 5.0f, g = 6.0f, h = 7.0f;
    __shared__ float lds[4096];
    lds[threadIdx.x & 4095] = a;
    __syncthreads();
    if (wave >= active_waves) return;  // after the only barrier
    unsigned va = (threadIdx.x & 63) * 4;
    uint64_t m = 0, m2 = 0;
    float m2f = 0.0f;
    if constexpr (K == 13) { a = (float)(threadIdx.x & 63); h = (float)active_lanes; }
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if constexpr (K == 0)  // 16 independent adds (8 regs, 2 rounds)
            asm volatile(REP8("v_add_f32 %0, %0, %1\n v_add_f32 %2, %2, %1\n v_add_f32 %3, %3, %1\n v_add_f32 %4, %4, %1\n"
                              "v_add_f32 %5, %5, %1\n v_add_f32 %6, %6, %1\n v_add_f32 %7, %7, %1\n v_add_f32 %8, %8, %1\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+v"(b));
        if constexpr (K == 1)  // 64 dependent adds
            asm volatile(REP16("v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
        if constexpr (K == 2)  // 64 dependent DPP adds (2 wait states provided by an independent add each)
            asm volatile(REP16("v_add_f32_dpp %0, |%0|, %1 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32 %2, %2, %1\n s_nop 0\n"
                               "v_add_f32_dpp %0, |%0|, %1 wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32 %2, %2, %1\n s_nop 0\n")
                         : "+v"(a), "+v"(b), "+v"(c));
        if constexpr (K == 3)  // 64 (v_cmp -> sgpr, s_or) pairs
            asm volatile(REP16("v_cmp_lt_f32_e64 %1, %0, %2\n s_or_b64 %3, %3, %1\n v_cmp_lt_f32_e64 %1, %2, %0\n s_or_b64 %3, %3, %1\n")
                         : "+v"(a), "=&s"(m), "+v"(b), "+s"(m2) : : "scc");
        if constexpr (K == 4)  // 64 independent v_cmp -> sgpr (no consumer)
            asm volatile(REP16("v_cmp_lt_f32_e64 %1, %0, %2\n v_cmp_lt_f32_e64 %3, %2, %0\n v_cmp_lt_f32_e64 %1, %0, %2\n v_cmp_lt_f32_e64 %3, %2, %0\n")
                         : "+v"(a), "=&s"(m), "+v"(b), "=&s"(m2));
        if constexpr (K == 5)  // 64 independent SALU
            asm volatile(REP16("s_or_b64 %0, %0, %1\n s_or_b64 %1, %1, %0\n s_or_b64 %0, %0, %1\n s_or_b64 %1, %1, %0\n") : "+s"(m), "+s"(m2) : : "scc");
        if constexpr (K == 6)  // 64 ds_min_f32 (no return), then one wait
            asm volatile(REP16("ds_min_f32 %0, %1\n ds_min_f32 %0, %1 offset:4\n ds_min_f32 %0, %1 offset:8\n ds_min_f32 %0, %1 offset:12\n") "s_waitcnt lgkmcnt(0)\n"
                         : "+v"(va) : "v"(a) : "memory");
        if constexpr (K == 7)  // 64 ds_read_b32 then wait
            asm volatile(REP16("ds_read_b32 %1, %0\n ds_read_b32 %2, %0 offset:4\n ds_read_b32 %3, %0 offset:8\n ds_read_b32 %4, %0 offset:12\n") "s_waitcnt lgkmcnt(0)\n"
                         : "+v"(va), "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : : "memory");
        if constexpr (K == 8)  // 64 independent v_min3
            asm volatile(REP16("v_min3_f32 %0, %1, %2, %3\n v_min3_f32 %4, %1, %2, %3\n v_min3_f32 %5, %1, %2, %3\n v_min3_f32 %6, %1, %2, %3\n")
                         : "=&v"(a), "+v"(b), "+v"(c), "+v"(d), "=&v"(e), "=&v"(f), "=&v"(g));
        if constexpr (K == 9)  // 64 dependent ds_read round trips
            asm volatile(REP16("ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n v_and_b32 %1, 0, %1\n v_add_u32 %0, %0, %1\n") : "+v"(va), "=&v"(a) : : "memory");
        if constexpr (K == 10)  // 64 v_add with abs on input (VOP3)
            asm volatile(REP16("v_add_f32_e64 %0, |%8|, %1\n v_add_f32_e64 %2, |%8|, %1\n v_add_f32_e64 %3, |%8|, %1\n v_add_f32_e64 %4, |%8|, %1\n")
                         : "=&v"(a), "+v"(b), "=&v"(c), "=&v"(d), "=&v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(h));
        if constexpr (K == 11)  // 64 independent v_add_f32_dpp
            asm volatile(REP16("v_add_f32_dpp %0, |%4|, %1 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %2, |%4|, %1 wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                               "v_add_f32_dpp %3, |%4|, %1 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %5, |%4|, %1 wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
                         : "=&v"(a), "+v"(b), "=&v"(c), "=&v"(d), "+v"(h), "=&v"(e));
        if constexpr (K == 13)  // 16 x (v_cmpx -> exec = lanes < n, ds_min, restore exec): 3 instr per unit
            asm volatile("s_mov_b64 %4, exec\n" REP16("v_cmpx_lt_f32_e64 %1, %2, %3\n s_nop 0\n ds_min_f32 %0, %3\n s_mov_b64 exec, %4\n") "s_waitcnt lgkmcnt(0)\n"
                         : "+v"(va), "=&s"(m), "+v"(a), "+v"(h), "=&s"(m2) : : "memory", "scc");
        if constexpr (K == 14)  // the CPL1 sweep step x16 (adds, 2 DPP, min3, ds_min, wait, minimum3, sub, ds_read, min)
            asm volatile(REP16("v_add_f32_e64 %1, |%0|, %4\n v_add_f32_dpp %2, |%0|, %5 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                               "v_add_f32_dpp %3, |%0|, %5 wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_min3_f32 %1, %1, %2, %3\n"
                               "ds_min_f32 %6, %1 offset:64\n s_waitcnt lgkmcnt(4)\n v_minimum3_f32 %0, %1, %7, %8\n v_sub_f32 %2, %1, %7\n"
                               "ds_read_b32 %7, %6 offset:128\n v_min_f32 %9, %2, %9\n") "s_waitcnt lgkmcnt(0)\n"
                         : "+v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "+v"(e), "+v"(f), "+v"(va), "+v"(g), "+v"(h), "+v"(m2f) : : "memory");
        if constexpr (K == 15)  // same without DPP (plain adds)
            asm volatile(REP16("v_add_f32_e64 %1, |%0|, %4\n v_add_f32_e64 %2, |%0|, %5\n"
                               "v_add_f32_e64 %3, |%0|, %5\n v_min3_f32 %1, %1, %2, %3\n"
                               "ds_min_f32 %6, %1 offset:64\n s_waitcnt lgkmcnt(4)\n v_minimum3_f32 %0, %1, %7, %8\n v_sub_f32 %2, %1, %7\n"
                               "ds_read_b32 %7, %6 offset:128\n v_min_f32 %9, %2, %9\n") "s_waitcnt lgkmcnt(0)\n"
                         : "+v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "+v"(e), "+v"(f), "+v"(va), "+v"(g), "+v"(h), "+v"(m2f) : : "memory");
        if constexpr (K == 16)  // same without LDS
            asm volatile(REP16("v_add_f32_e64 %1, |%0|, %4\n v_add_f32_dpp %2, |%0|, %5 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                               "v_add_f32_dpp %3, |%0|, %5 wave_rol:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_min3_f32 %1, %1, %2, %3\n"
                               "v_minimum3_f32 %0, %1, %7, %8\n v_sub_f32 %2, %1, %7\n"
                               "v_min_f32 %9, %2, %9\n")
                         : "+v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "+v"(e), "+v"(f), "+v"(va), "+v"(g), "+v"(h), "+v"(m2f) : : "memory");
        if constexpr (K == 12)  // 64 v_pk_add_f32
            asm volatile(REP16("v_pk_add_f32 %0, %1, %2\n v_pk_add_f32 %3, %1, %2\n v_pk_add_f32 %4, %1, %2\n v_pk_add_f32 %5, %1, %2\n")
                         : "=&v"(*(double*)&m), "+v"(*(double*)&m2), "+v"(*(double*)&va), "=&v"(*(double*)&a), "=&v"(*(double*)&c), "=&v"(*(double*)&e));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) out[wave] = t1 - t0;
    if (threadIdx.x == 0) out[63] = (unsigned long long)(a + b + c + d + e + f + g + h + m2f + (float)m + (float)m2 + (float)va);
}

template <int K>
void run(const char *name, unsigned long long *d, int waves, int lanes = 64)
{
    unsigned long long h[64];
    const int iters = 200;
    fprintf(stderr, "start %s %d\n", name, waves);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(bench<K>, dim3(1), dim3(1024), 0, 0, d, iters, waves, lanes);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-28s waves=%2d lanes=%2d %.2f cycles/instr (wave0)\n", name, waves, lanes, (double)h[0] / (iters * 64.0));
    fflush(stdout);
}

int main()
{
    unsigned long long *d;
    hipMalloc(&d, 64 * 8);
    for (int w : {1, 2, 4, 8, 16}) {
        run<14>("CPL1 step x16 (per instr, 10/step)", d, w);
        run<15>("CPL1 step no DPP", d, w);
        run<16>("CPL1 step no LDS (7/step)", d, w);
    }
    return 0;
}
