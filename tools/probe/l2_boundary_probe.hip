// Does data a kernel wrote stay usable in its XCD's L2 for the NEXT kernel on the same stream?
// Kernel W: the workgroups that run on XCD `xw` (read from HW_REG_XCC_ID) write a 1 MiB buffer with
// plain stores, 32 KiB per workgroup slot.  Kernel R (next launch): the workgroups on XCD `xr` read
// the same slots and time their loads (s_memrealtime, 10 ns ticks).  xr == xw vs xr != xw: same-XCD
// L2 retention across the kernel boundary.  Also R after a 512 MiB streaming kernel (cold).
// Build: hipcc --offload-arch=gfx950 -O3 -o l2_boundary_probe l2_boundary_probe.hip ; run: ./l2_boundary_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ int xcd_slot(unsigned *cnt, int *xo)
{
    __shared__ int sh[2];
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        x &= 7u;
        sh[0] = (int)x;
        sh[1] = (int)__hip_atomic_fetch_add(cnt + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    *xo = sh[0];
    return sh[1];
}

constexpr int SLOTS = 32, SLOT_F4 = 32 * 1024 / 16;   // 32 slots x 32 KiB = 1 MiB

__global__ __launch_bounds__(256) void k_write(unsigned *cnt, f32x4 *buf, int xw, float v)
{
    int x;
    const int slot = xcd_slot(cnt, &x);
    if (x != xw || slot >= SLOTS) return;
    f32x4 *p = buf + (size_t)slot * SLOT_F4;
    for (int i = threadIdx.x; i < SLOT_F4; i += 256) p[i] = f32x4{v, v + 1, v + 2, v + 3};
}

__global__ __launch_bounds__(256) void k_read(unsigned *cnt, const f32x4 *buf, int xr, unsigned *ticks, float *sink)
{
    int x;
    const int slot = xcd_slot(cnt, &x);
    if (x != xr || slot >= SLOTS) return;
    const f32x4 *p = buf + (size_t)slot * SLOT_F4;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    f32x4 acc = {0, 0, 0, 0};
    f32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[threadIdx.x + 256 * k];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) ticks[slot] = (unsigned)(t1 - t0);
    if (acc.x == -1.0f) sink[0] = acc.y;
}

__global__ __launch_bounds__(256) void k_stream(f32x4 *big, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        big[i] = big[i] + f32x4{1, 1, 1, 1};
}

int main()
{
    unsigned *cnt, *ticks;
    f32x4 *buf, *big;
    float *sink;
    const size_t nbig = (size_t)512 << 20 >> 4;
    hipMalloc(&cnt, 64);
    hipMalloc(&ticks, 4 * SLOTS);
    hipMalloc(&buf, 1 << 20);
    hipMalloc(&big, nbig * 16);
    hipMalloc(&sink, 4);
    hipMemset(big, 0, nbig * 16);
    std::vector<unsigned> h(SLOTS);
    auto run = [&](const char *name, int xw, int xr, bool cold) {
        std::vector<double> med;
        for (int rep = 0; rep < 9; ++rep) {
            hipMemset(cnt, 0, 64);
            hipLaunchKernelGGL(k_write, dim3(2048), dim3(256), 0, 0, cnt, buf, xw, (float)rep);
            if (cold) hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, big, nbig);
            hipMemset(cnt, 0, 64);
            hipMemset(ticks, 0, 4 * SLOTS);
            hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, cnt, buf, xr, ticks, sink);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), ticks, 4 * SLOTS, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.end());
            med.push_back(h[SLOTS / 2] * 10.0);   // ns
        }
        std::sort(med.begin(), med.end());
        printf("%-34s read 32 KiB per workgroup: median %.0f ns (min %.0f, max %.0f over reps)\n", name, med[4],
               med[0], med[8]);
    };
    run("same XCD as the writer", 0, 0, false);
    run("other XCD", 0, 1, false);
    run("same XCD, 512 MiB stream between", 0, 0, true);
    run("same XCD (xcd 3)", 3, 3, false);
    run("other XCD (3 -> 6)", 3, 6, false);
    return 0;
}
