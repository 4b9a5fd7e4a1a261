// Repro: does a replayed hipGraph kernel node see the kernel-argument bytes it was captured with?
// Each of NL launches writes its by-value argument tail (w[8], idx) into out; the graph is replayed
// several times and every replay's out is compared with the direct-launch result.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

template <int PAD>
struct Args {
    const float *src;
    char pad[PAD];
    int idx;
    float w[8];
};

template <int PAD>
__global__ void k(Args<PAD> a, float *out)
{
    const int t = threadIdx.x;
    if (t < 8) out[a.idx * 9 + t] = a.w[t] + a.src[0];
    if (t == 8) out[a.idx * 9 + 8] = (float)a.pad[PAD - 1];
}

template <int PAD>
int run(int NL, int reps)
{
    float *src, *out;
    (void)hipMalloc(&src, 4);
    (void)hipMemset(src, 0, 4);
    (void)hipMalloc(&out, NL * 9 * 4);
    hipStream_t s, cap;
    (void)hipStreamCreate(&s);
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    auto launch_all = [&](hipStream_t st) {
        Args<PAD> a{};
        a.src = src;
        for (int i = 0; i < NL; ++i) {
            a.idx = i;
            a.pad[PAD - 1] = (char)(i & 127);
            for (int t = 0; t < 8; ++t) a.w[t] = 1000.0f * i + t;
            hipLaunchKernelGGL(k<PAD>, dim3(1), dim3(64), 0, st, a, out);
        }
    };
    std::vector<float> ref(NL * 9), got(NL * 9);
    (void)hipMemsetAsync(out, 0, NL * 9 * 4, s);
    launch_all(s);
    (void)hipMemcpyAsync(ref.data(), out, NL * 9 * 4, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    hipGraph_t g;
    (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    launch_all(cap);
    (void)hipStreamEndCapture(cap, &g);
    hipGraphExec_t ex;
    (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    int bad_total = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemsetAsync(out, 0, NL * 9 * 4, s);
        (void)hipGraphLaunch(ex, s);
        (void)hipMemcpyAsync(got.data(), out, NL * 9 * 4, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        int bad = 0, first = -1;
        for (int i = 0; i < NL * 9; ++i)
            if (memcmp(&got[i], &ref[i], 4)) { if (first < 0) first = i; ++bad; }
        printf("{\"pad\": %d, \"argbytes\": %zu, \"launches\": %d, \"rep\": %d, \"bad\": %d, \"first\": %d, \"got\": %g, \"want\": %g}\n",
               PAD, sizeof(Args<PAD>), NL, r, bad, first, first >= 0 ? got[first] : 0.0f, first >= 0 ? ref[first] : 0.0f);
        bad_total += bad;
    }
    (void)hipGraphExecDestroy(ex);
    (void)hipFree(src); (void)hipFree(out);
    (void)hipStreamDestroy(s); (void)hipStreamDestroy(cap);
    return bad_total;
}

// Memset nodes: a captured hipMemsetAsync of `bytes` followed by a kernel that accumulates into the
// zeroed region (out[i] += 1); every replay must leave exactly 1 in each element.
__global__ void kacc(float *out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] += 1.0f;
}

int run_memset(size_t bytes, int reps)
{
    const int n = (int)(bytes / 4);
    float *buf;
    (void)hipMalloc(&buf, bytes);
    hipStream_t s, cap;
    (void)hipStreamCreate(&s);
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    hipGraph_t g;
    (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    (void)hipMemsetAsync(buf, 0, bytes, cap);
    hipLaunchKernelGGL(kacc, dim3((n + 255) / 256), dim3(256), 0, cap, buf, n);
    (void)hipStreamEndCapture(cap, &g);
    hipGraphExec_t ex;
    (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    std::vector<float> h(n);
    int bad_total = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipGraphLaunch(ex, s);
        (void)hipMemcpyAsync(h.data(), buf, bytes, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        int bad = 0;
        for (int i = 0; i < n; ++i) bad += h[i] != 1.0f;
        printf("{\"memset_bytes\": %zu, \"rep\": %d, \"bad\": %d, \"v0\": %g}\n", bytes, r, bad, h[0]);
        bad_total += bad;
    }
    (void)hipGraphExecDestroy(ex);
    (void)hipFree(buf);
    (void)hipStreamDestroy(s); (void)hipStreamDestroy(cap);
    return bad_total;
}

// Stream order: a slow kernel fills the buffer with NaN on stream `s`, then the captured graph
// (memset 0 + out[i] += 1) is launched on the same stream.  Every element must end at exactly 1.
__global__ void kslow_fill(float *out, int n, int spins)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float x = 0.0f;
    for (int k = 0; k < spins; ++k) x = x * 0.999f + 1.0f;   // ~spins x 4 cycles of dependent FMAs
    if (i < n) out[i] = __builtin_nanf("") + x * 0.0f;
}

int run_order(int which, size_t bytes, int spins, int reps)
{
    const int n = (int)(bytes / 4);
    float *buf;
    (void)hipMalloc(&buf, bytes);
    hipStream_t s = nullptr, cap;
    if (which == 1) (void)hipStreamCreate(&s);
    if (which == 2) s = hipStreamPerThread;
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    hipGraph_t g;
    (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    (void)hipMemsetAsync(buf, 0, bytes, cap);
    hipLaunchKernelGGL(kacc, dim3((n + 255) / 256), dim3(256), 0, cap, buf, n);
    (void)hipStreamEndCapture(cap, &g);
    hipGraphExec_t ex;
    (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    (void)hipDeviceSynchronize();
    std::vector<float> h(n);
    int bad_total = 0;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(kslow_fill, dim3((n + 255) / 256), dim3(256), 0, s, buf, n, spins);
        (void)hipGraphLaunch(ex, s);
        (void)hipMemcpyAsync(h.data(), buf, bytes, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        int bad = 0;
        for (int i = 0; i < n; ++i) bad += h[i] != 1.0f;
        printf("{\"order_stream\": \"%s\", \"bytes\": %zu, \"spins\": %d, \"rep\": %d, \"bad\": %d, \"v0\": %g}\n",
               which == 0 ? "null" : which == 1 ? "created" : "per_thread", bytes, spins, r, bad, h[0]);
        bad_total += bad;
    }
    (void)hipGraphExecDestroy(ex);
    (void)hipFree(buf);
    if (which == 1) (void)hipStreamDestroy(s);
    (void)hipStreamDestroy(cap);
    return bad_total;
}

// memset node + NK kernel nodes (each out[i] += 1 over the zeroed region): every replay must end at NK.
// fill: the buffer is set to 0xFF bytes (NaN) with a plain hipMemset before every launch.
int run_memset_chain(size_t bytes, int NK, int reps, bool fill)
{
    const int n = (int)(bytes / 4);
    float *buf;
    (void)hipMalloc(&buf, bytes);
    hipStream_t s, cap;
    (void)hipStreamCreate(&s);
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    hipGraph_t g;
    (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    (void)hipMemsetAsync(buf, 0, bytes, cap);
    for (int k = 0; k < NK; ++k) hipLaunchKernelGGL(kacc, dim3((n + 255) / 256), dim3(256), 0, cap, buf, n);
    (void)hipStreamEndCapture(cap, &g);
    hipGraphExec_t ex;
    (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    std::vector<float> h(n);
    int bad_total = 0;
    for (int r = 0; r < reps; ++r) {
        if (fill) { (void)hipMemset(buf, 0xFF, bytes); (void)hipDeviceSynchronize(); }
        (void)hipGraphLaunch(ex, s);
        (void)hipMemcpyAsync(h.data(), buf, bytes, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        int bad = 0;
        for (int i = 0; i < n; ++i) bad += h[i] != (float)NK;
        printf("{\"chain_bytes\": %zu, \"kernels\": %d, \"fill\": %d, \"rep\": %d, \"bad\": %d, \"v0\": %g}\n", bytes, NK,
               (int)fill, r, bad, h[0]);
        bad_total += bad;
    }
    (void)hipGraphExecDestroy(ex);
    (void)hipFree(buf);
    (void)hipStreamDestroy(s); (void)hipStreamDestroy(cap);
    return bad_total;
}

int main()
{
    int bad = 0;
    for (int nk : {1, 2, 8, 50})
        for (bool fill : {false, true}) bad += run_memset_chain(40960, nk, 3, fill);
    for (int which : {0, 1, 2})
        for (int spins : {1000, 100000}) bad += run_order(which, 40960, spins, 3);
    for (size_t b : {4, 8, 16, 32, 64, 128, 256, 4096, 40960, 1 << 20}) bad += run_memset(b, 3);
    for (int nl : {4, 40, 200}) {
        bad += run<16>(nl, 3);
        bad += run<200>(nl, 3);
        bad += run<400>(nl, 3);
        bad += run<1000>(nl, 3);
    }
    printf("{\"total_bad\": %d}\n", bad);
    return 0;
}
