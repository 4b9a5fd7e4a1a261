// Same-XCD hand-off probe: which store / load cache-policy pairs make a granule written by one
// workgroup visible to another workgroup on the SAME XCD (read from HW_REG_XCC_ID), and how fast.
// Per XCD: slot 0 = producer, slot 1 = consumer; ping-pong of 8-byte {value, tag} granules.
// Build: hipcc --offload-arch=gfx950 -O3 -o l2_probe l2_probe.hip ; run: ./l2_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int SP, int LP>
__global__ void k_probe(unsigned *cnt, unsigned long long *gran, unsigned *res, int iters, int cross)
{
    __shared__ int sh[2];
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        x &= 7u;
        const unsigned slot = __hip_atomic_fetch_add(cnt + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned tot = 0;
        do {
            tot = 0;
            for (int i = 0; i < 8; ++i) tot += __hip_atomic_load(cnt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } while (tot < gridDim.x);
        sh[0] = (int)x; sh[1] = (int)slot;
    }
    __syncthreads();
    const int x = sh[0], slot = sh[1];
    // cross = 0: pair inside XCD x (slots 0 / 1); cross = 1: producer on XCD x, consumer on XCD x^1
    int role = -1, pair = x;
    if (!cross) { if (slot == 0) role = 0; else if (slot == 1) role = 1; }
    else { if (slot == 0 && (x & 1) == 0) role = 0; if (slot == 0 && (x & 1) == 1) { role = 1; pair = x ^ 1; } }
    if (role < 0 || threadIdx.x != 0) return;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(gran + pair * 64, (short)0, 0x7fffffff, 0x00020000);
    const int my = role == 0 ? 0 : 32 * 8, other = role == 0 ? 32 * 8 : 0;   // separate 256-B lines
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned fails = 0;
    for (int e = 1; e <= iters; ++e) {
        if (role == 1 || e > 1) {       // wait for the other side's tag (producer waits for the ack)
            const unsigned want = role == 1 ? (unsigned)e : (unsigned)(e - 1);
            const unsigned long long ts = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, other, 0, LP);
                if (v.y == want) break;
                if (__builtin_amdgcn_s_memrealtime() - ts > 2000000ull) { fails++; break; }   // 20 ms
            }
        }
        if (fails > 3) break;
        u32x2 o; o.x = e; o.y = e;
        __builtin_amdgcn_raw_buffer_store_b64(o, rs, my, 0, SP);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    res[pair * 4 + role * 2 + 0] = (unsigned)(t1 - t0);
    res[pair * 4 + role * 2 + 1] = fails;
}

template <int SP, int LP>
void run(const char *name, int cross, unsigned *cnt, unsigned long long *gran, unsigned *res)
{
    const int iters = 2000;
    for (int rep = 0; rep < 3; ++rep) {
        hipMemset(cnt, 0, 64);
        hipMemset(res, 0, 256);
        if (rep == 2) {   // dirty the granule lines from other XCDs first (plain stores everywhere)
            hipMemset(gran, 0xff, 8 * 64 * 8);
        } else {
            hipMemset(gran, 0, 8 * 64 * 8);
        }
        hipLaunchKernelGGL((k_probe<SP, LP>), dim3(256), dim3(64), 0, 0, cnt, gran, res, iters, cross);
        hipDeviceSynchronize();
        std::vector<unsigned> h(64);
        hipMemcpy(h.data(), res, 256, hipMemcpyDeviceToHost);
        double us = 0; unsigned f = 0; int n = 0;
        for (int p = 0; p < 8; ++p) { if (h[p * 4]) { us += h[p * 4] * 0.01; n++; } f += h[p * 4 + 1] + h[p * 4 + 3]; }
        printf("%-28s cross=%d rep=%d  round trip %.3f us  fails %u\n", name, cross, rep, n ? us / n / iters : -1.0, f);
    }
}

int main()
{
    unsigned *cnt, *res;
    unsigned long long *gran;
    hipMalloc(&cnt, 64); hipMalloc(&res, 256); hipMalloc(&gran, 8 * 64 * 8);
    for (int cross = 0; cross < 2; ++cross) {
        run<16, 16>("store sc1 / load sc1", cross, cnt, gran, res);
        run<0, 16>("store plain / load sc1", cross, cnt, gran, res);
        run<0, 2>("store plain / load nt", cross, cnt, gran, res);
        run<0, 17>("store plain / load sc0sc1", cross, cnt, gran, res);
        run<1, 1>("store sc0 / load sc0", cross, cnt, gran, res);
        run<0, 1>("store plain / load sc0", cross, cnt, gran, res);
    }
    return 0;
}
