// relu_stream.hip -- what bounds the rectify backward's stream rate (csr_ops.hip
// relu_backward_kernel: read g + gate bytes, write g, per-column sums) at 1.4 M x 300 (row
// stride 304 floats, gate stride 300 B)? Variants, each timed with hipEvents (mean of 20):
//   flat   : float4 copy of the whole padded g matrix, grid-stride (the achievable stream rate)
//   rowcp  : the kernel's mapping (wave = one row per step, lane = float4 columns l, l + 64),
//            copy only (no gate, no sums)
//   rowgate: + gate bytes, masked store (no sums)
//   full   : + per-lane column sums (the kernel as it is)
//   full_b : full with 4096 workgroups instead of 1024
// Build: hipcc --offload-arch=gfx950 -O3 -o relu_stream relu_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void flat_copy(int64_t n4, const float4* __restrict__ a,
                                                 float4* __restrict__ b) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride)
    b[i] = a[i];
}

__device__ __forceinline__ float gate_apply(float g, uint32_t code) {
  return code == 2u ? g : (code == 1u ? 0.5f * g : 0.0f);
}

template <int MODE>  // 0 copy, 1 gate, 2 gate + sums
__global__ __launch_bounds__(256) void rows_kernel(int64_t M, int K, int64_t rpb, const float* g,
                                                   int64_t ldg, const uint8_t* __restrict__ gate,
                                                   int64_t ldgate, float* out, int64_t ldo,
                                                   float* __restrict__ partial) {
  __shared__ float red[4][4 * 64 * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rpb;
  const int64_t r1 = min(M, r0 + rpb);
  const int pieces = (K + 255) / 256;
  float acc[4][4] = {};
#pragma unroll 2
  for (int64_t r = r0 + w; r < r1; r += 4) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p >= pieces) break;
      const int c = (p * 64 + lane) * 4;
      if (c + 4 > K) continue;
      float4 o = *reinterpret_cast<const float4*>(g + r * ldg + c);
      if constexpr (MODE >= 1) {
        const uint32_t t = *reinterpret_cast<const uint32_t*>(gate + r * ldgate + c);
        o = make_float4(gate_apply(o.x, t & 0xffu), gate_apply(o.y, (t >> 8) & 0xffu),
                        gate_apply(o.z, (t >> 16) & 0xffu), gate_apply(o.w, t >> 24));
      }
      *reinterpret_cast<float4*>(out + r * ldo + c) = o;
      if constexpr (MODE == 2) {
        acc[p][0] += o.x; acc[p][1] += o.y; acc[p][2] += o.z; acc[p][3] += o.w;
      }
    }
  }
  if constexpr (MODE == 2) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w][(p * 64 + lane) * 4 + e] = acc[p][e];
    __syncthreads();
    for (int c = threadIdx.x; c < K; c += 256)
      partial[static_cast<int64_t>(blockIdx.x) * K + c] =
          ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
  }
}

int main() {
  const int64_t M = 1400000;
  const int K = 300, ldg = 304, ldgate = 300;
  float *g, *o, *part;
  uint8_t* gate;
  CK(hipMalloc(&g, sizeof(float) * M * ldg));
  CK(hipMalloc(&o, sizeof(float) * M * ldg));
  CK(hipMalloc(&gate, M * ldgate));
  CK(hipMalloc(&part, sizeof(float) * 8192 * K));
  CK(hipMemset(g, 0x3f, sizeof(float) * M * ldg));
  CK(hipMemset(gate, 2, M * ldgate));
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  auto timeit = [&](const char* name, double bytes, auto&& launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(s));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, s, e));
    ms /= 20;
    std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, bytes / ms / 1e9);
  };
  const double gbytes = 8.0 * M * K, gate_bytes = 1.0 * M * K;
  const int64_t n4 = M * ldg / 4;
  for (int blocks : {1024, 2048, 4096, 8192}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "flat_%d", blocks);
    timeit(nm, 8.0 * M * ldg, [&] {
      hipLaunchKernelGGL(flat_copy, dim3(blocks), dim3(256), 0, 0, n4,
                         reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(o));
    });
  }
  for (int nb : {1024, 2048, 4096, 8192}) {
    const int64_t r = (M + nb - 1) / nb;
    const int64_t rpb = (r + 3) / 4 * 4;
    const int64_t grid = (M + rpb - 1) / rpb;
    char nm[64];
    std::snprintf(nm, sizeof nm, "rowcp_%d", nb);
    timeit(nm, gbytes, [&] {
      hipLaunchKernelGGL(rows_kernel<0>, dim3(grid), dim3(256), 0, 0, M, K, rpb, g, int64_t(ldg),
                         gate, int64_t(ldgate), o, int64_t(ldg), part);
    });
    std::snprintf(nm, sizeof nm, "rowgate_%d", nb);
    timeit(nm, gbytes + gate_bytes, [&] {
      hipLaunchKernelGGL(rows_kernel<1>, dim3(grid), dim3(256), 0, 0, M, K, rpb, g, int64_t(ldg),
                         gate, int64_t(ldgate), o, int64_t(ldg), part);
    });
    std::snprintf(nm, sizeof nm, "full_%d", nb);
    timeit(nm, gbytes + gate_bytes, [&] {
      hipLaunchKernelGGL(rows_kernel<2>, dim3(grid), dim3(256), 0, 0, M, K, rpb, g, int64_t(ldg),
                         gate, int64_t(ldgate), o, int64_t(ldg), part);
    });
  }
  CK(hipDeviceSynchronize());
  std::printf("done\n");
  return 0;
}
