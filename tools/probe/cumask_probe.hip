// Which XCD does each CU-mask bit select?  For every CU i a stream with only bit i of the CU mask set
// (hipExtStreamCreateWithCUMask) runs 64 one-wave workgroups that record HW_REG_XCC_ID; prints
// "cu <i>: xcd <x> (<n> workgroups) per-xcd <8 counts>".
// Build: hipcc --offload-arch=gfx950 -O3 -o cumask_probe cumask_probe.hip ; run: ./cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

__global__ void k_xcc(unsigned *out)
{
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        __hip_atomic_fetch_add(out + (x & 7u), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main()
{
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    printf("CUs %d\n", cus);
    unsigned *d_out = nullptr;
    hipMalloc(&d_out, 8 * sizeof(unsigned));
    const int words = (cus + 31) / 32;
    for (int i = 0; i < cus; ++i) {
        std::vector<uint32_t> mask(words, 0u);
        mask[i / 32] |= 1u << (i % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, words, mask.data()) != hipSuccess) { printf("cu %d: create failed\n", i); continue; }
        hipMemsetAsync(d_out, 0, 8 * sizeof(unsigned), s);
        hipLaunchKernelGGL(k_xcc, dim3(64), dim3(64), 0, s, d_out);
        unsigned h[8];
        hipMemcpyAsync(h, d_out, sizeof(h), hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        int n = 0, x = -1, nx = 0;
        for (int k = 0; k < 8; ++k) if (h[k]) { n += h[k]; x = k; ++nx; }
        printf("cu %d: xcd %d (%d workgroups%s) per-xcd %u %u %u %u %u %u %u %u\n", i, x, n, nx > 1 ? ", several XCDs" : "",
               h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
        hipStreamDestroy(s);
    }
    hipFree(d_out);
    return 0;
}
