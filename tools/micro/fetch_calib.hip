// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths of the ingest kernels
// (/opt/skills/guides/MI355X_MICROARCH.md: only 16-B-per-lane streaming reads and stores are
// calibrated on gfx950; "calibrate on a known byte count in your own access pattern").
// Each kernel touches exactly BYTES bytes of a buffer larger than the 256 MiB Infinity Cache:
//   read16  16 B per lane, coalesced            (the point pass's depth / seg loads)
//   read8   8 B per lane, coalesced             (the resolve's key loads)
//   write8  8 B per lane, coalesced             (the resolve's key zeroing)
//   write4  4 B per lane, coalesced             (the resolve's overhead stores)
//   amax8   64-bit atomicMax per lane, coalesced (the point pass's key flush)
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/fetch_calib.hip -o /tmp/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE -- /tmp/fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- /tmp/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t BYTES = (size_t)512 << 20;

__global__ void read16(const uint4 *p, size_t n, unsigned *sink)
{
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc.x ^= v.x, acc.y ^= v.y, acc.z ^= v.z, acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345679u) sink[0] = 1;
}
__global__ void read8(const unsigned long long *p, size_t n, unsigned *sink)
{
    unsigned long long acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i];
    if (acc == 0x123456789ull) sink[0] = 1;
}
__global__ void write8(unsigned long long *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0ull;
}
__global__ void write4(float *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0.5f;
}
__global__ void amax8(unsigned long long *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        atomicMax(&p[i], (unsigned long long)i);
}

int main()
{
    void *buf = nullptr;
    unsigned *sink = nullptr;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    if (hipMemset(buf, 0, BYTES) != hipSuccess) return 1;
    const dim3 g(4096), b(256);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(read16, g, b, 0, 0, (const uint4 *)buf, BYTES / 16, sink);
        hipLaunchKernelGGL(read8, g, b, 0, 0, (const unsigned long long *)buf, BYTES / 8, sink);
        hipLaunchKernelGGL(write8, g, b, 0, 0, (unsigned long long *)buf, BYTES / 8);
        hipLaunchKernelGGL(write4, g, b, 0, 0, (float *)buf, BYTES / 4);
        hipLaunchKernelGGL(amax8, g, b, 0, 0, (unsigned long long *)buf, BYTES / 8);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes_per_kernel\": %zu}\n", BYTES);
    (void)hipFree(buf);
    (void)hipFree(sink);
    return 0;
}
