"""Timing-only build of the bf16 halo-staged conv with per-workgroup phase stamps (never shipped): entry (t0),
chunk 0 staged + first barrier (t1), every chunk's taps done (t2), epilogue done (t3), s_memrealtime (10 ns),
stored by thread 0 of each workgroup into a device array read by rdq_exp_c3prof.  Output:
red-diffeq_amd/lib_exp/libc3prof.so (RDQ_HIP_LIB selects it; tools/c3_phase.py reads the stamps)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "red-diffeq_amd")
src = open(os.path.join(PKG, "csrc", "unet.hip")).read()


def once(old, new):
    global src
    i = src.index(old)
    src = src[:i] + new + src[i + len(old):]


once("template <int MODE, bool IN8 = false>\n__global__ __launch_bounds__(256, 2) void k_conv3_bf16(C3Args a)\n{",
     "__device__ unsigned long long g_c3p[4 * 65536];\n"
     "template <int MODE, bool IN8 = false>\n__global__ __launch_bounds__(256, 2) void k_conv3_bf16(C3Args a)\n{\n"
     "    const unsigned long long c3t0 = __builtin_amdgcn_s_memrealtime();")
once("    wstash(0, wr[0]);\n    __syncthreads();\n",
     "    wstash(0, wr[0]);\n    __syncthreads();\n    const unsigned long long c3t1 = __builtin_amdgcn_s_memrealtime();\n")
once("    chunk(a.cch - 1, std::false_type{});\n",
     "    chunk(a.cch - 1, std::false_type{});\n    const unsigned long long c3t2 = __builtin_amdgcn_s_memrealtime();\n")
once("    c3_epilogue(a, acc, pl, &Hs[0][0][0], c3g);\n",
     "    c3_epilogue(a, acc, pl, &Hs[0][0][0], c3g);\n"
     "    if (threadIdx.x == 0) {\n"
     "        const size_t i_ = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) & 65535;\n"
     "        g_c3p[4 * i_] = c3t0; g_c3p[4 * i_ + 1] = c3t1; g_c3p[4 * i_ + 2] = c3t2;\n"
     "        g_c3p[4 * i_ + 3] = __builtin_amdgcn_s_memrealtime();\n"
     "    }\n")
i = src.rindex("}  // extern \"C\"")
src = src[:i] + ("int rdq_exp_c3prof(void *out, int n)\n{\n"
                 "    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c3p), (size_t)n * 32) != hipSuccess) return -1;\n"
                 "    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;\n}\n\n") + src[i:]
os.makedirs("/tmp/exp", exist_ok=True)
open("/tmp/exp/unet_c3prof.hip", "w").write(src)
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                       "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"), "-c", "-o",
                       "/tmp/exp/unet_c3prof.o", "/tmp/exp/unet_c3prof.hip"])
os.makedirs(os.path.join(PKG, "lib_exp"), exist_ok=True)
out = os.path.join(PKG, "lib_exp", "libc3prof.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", out, "/tmp/exp/unet_c3prof.o",
                       os.path.join(PKG, "build", "fwi.o"), os.path.join(PKG, "build", "loop.o")])
print(out)
