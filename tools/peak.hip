// Roofline calibration on the box ("to be confirmed on the box by an MFMA microbenchmark"):
//   * bf16 MFMA: every CU, one wave per SIMD, back-to-back v_mfma_f32_32x32x16_bf16 on random operands
//     (4 independent accumulators per wave), timed with HIP events -> dense TFLOP/s at the clock held under load;
//   * HBM read: a 4 GiB buffer read once with 16-B loads (grid-stride, 8 loads in flight per thread);
//   * HBM copy: 2 GiB -> 2 GiB (read + write bytes counted).
// Build: hipcc --offload-arch=gfx950 -O3 tools/peak.hip -o tools/peak   Run: tools/peak  (prints one JSON line)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

constexpr int MF_ITERS = 16384;  // 4 MFMAs per iteration

__global__ __launch_bounds__(256) void mfma_peak_kernel(const bf16x8* __restrict__ src, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  bf16x8 a = src[lane], b = src[64 + lane];
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < MF_ITERS; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += c0[e] + c1[e] + c2[e] + c3[e];
  out[blockIdx.x * 256 + threadIdx.x] = s;  // keeps the chain live
}

__global__ __launch_bounds__(256) void hbm_read_kernel(const u32x4* __restrict__ p, long long n, unsigned* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  unsigned acc = 0;
  for (; i + 7 * stride < n; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  for (; i < n; i += stride) {
    const u32x4 v = p[i];
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void hbm_copy_kernel(const u32x4* __restrict__ p, u32x4* __restrict__ q, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[i + u * stride] = v[u];
  }
  for (; i < n; i += stride) q[i] = p[i];
}

template <typename F>
static float best_ms(F&& launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();  // warm-up
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return best;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;

  // MFMA: one 256-thread workgroup (4 waves: one per SIMD) per CU
  std::vector<unsigned short> h(128 * 8);
  unsigned st = 12345u;
  for (auto& v : h) {
    st = st * 1664525u + 1013904223u;
    v = (unsigned short)(0x3c00u + ((st >> 16) & 0x7fu));  // bf16 values in [0.0078, 0.0156): finite sums
  }
  bf16x8* src;
  float* out;
  CK(hipMalloc(&src, h.size() * 2));
  CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)ncu * 256 * 4));
  const float ms_mfma = best_ms([&] { hipLaunchKernelGGL(mfma_peak_kernel, dim3(ncu), dim3(256), 0, 0, src, out); }, 10);
  CK(hipGetLastError());
  const double flops = (double)ncu * 4 * MF_ITERS * 4 * 2.0 * 32 * 32 * 16;

  const long long bytes = 4LL << 30;
  u32x4 *buf, *dst;
  unsigned* ro;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  CK(hipMalloc(&ro, (size_t)ncu * 8 * 256 * 4));
  const long long n16 = bytes / 16;
  const float ms_read =
      best_ms([&] { hipLaunchKernelGGL(hbm_read_kernel, dim3(ncu * 8), dim3(256), 0, 0, buf, n16, ro); }, 10);
  CK(hipGetLastError());
  dst = buf + n16 / 2;  // copy the first 2 GiB into the second
  const float ms_copy =
      best_ms([&] { hipLaunchKernelGGL(hbm_copy_kernel, dim3(ncu * 8), dim3(256), 0, 0, buf, dst, n16 / 2); }, 10);
  CK(hipGetLastError());
  printf("{\"device\": \"%s\", \"cus\": %d, \"mfma_bf16_dense_tflops\": %.1f, \"mfma_ms\": %.4f, "
         "\"hbm_read_gbs\": %.0f, \"hbm_copy_gbs\": %.0f, \"read_bytes\": %lld, \"copy_bytes\": %lld}\n",
         prop.gcnArchName, ncu, flops / (ms_mfma * 1e-3) / 1e12, ms_mfma, bytes / (ms_read * 1e-3) / 1e9,
         bytes / (ms_copy * 1e-3) / 1e9, bytes, bytes);
  CK(hipFree(src));
  CK(hipFree(out));
  CK(hipFree(buf));
  CK(hipFree(ro));
  return 0;
}
