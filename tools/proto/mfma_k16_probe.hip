// Round 5 probe: cycles per v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16 on gfx950
// (one wave per SIMD, 4 independent accumulators, random-ish operands), and whether the
// 16-deep form on the low k half equals the 32-deep form with the high k half zero (bitwise).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
using bf8 = __attribute__((ext_vector_type(8))) __bf16;
using bf4 = __attribute__((ext_vector_type(4))) __bf16;
using f4 = __attribute__((ext_vector_type(4))) float;

template <int K32>
__global__ void loop_kernel(float* out, long long* cyc, int iters, float seed) {
  const int l = threadIdx.x & 63;
  bf8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(seed * (l + 1) * (i + 3) * 0.001f);
    b[i] = (__bf16)(seed * (l + 7) * (i + 1) * 0.0013f);
  }
  const bf4 a4 = {a[0], a[1], a[2], a[3]}, b4 = {b[0], b[1], b[2], b[3]};
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (K32) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c3, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  const f4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// bitwise: acc += A.B over k < 16 with both forms (the 32-deep one with k >= 16 zero), from
// random operands and a random starting accumulator
__global__ void eq_kernel(const float* r, int* bad) {
  const int l = threadIdx.x;
  bf8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = i < 4 ? (__bf16)r[l * 16 + i] : (__bf16)0.f;
    b[i] = i < 4 ? (__bf16)r[l * 16 + 8 + i] : (__bf16)0.f;
  }
  const bf4 a4 = {a[0], a[1], a[2], a[3]}, b4 = {b[0], b[1], b[2], b[3]};
  f4 c = {r[1024 + l], r[1088 + l], r[1152 + l], r[1216 + l]};
  f4 x = c, y = c;
  for (int it = 0; it < 64; ++it) {
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, x, 0, 0, 0);
    y = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, y, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i)
    if (__builtin_bit_cast(unsigned, x[i]) != __builtin_bit_cast(unsigned, y[i])) atomicAdd(bad, 1);
}

int main() {
  float* out; long long* cyc; int* bad; float* r;
  const int blocks = 1024, iters = 4096;
  hipMalloc(&out, blocks * 256 * 4); hipMalloc(&cyc, blocks * 8); hipMalloc(&bad, 4); hipMalloc(&r, 2048 * 4);
  float hr[2048]; unsigned s = 12345;
  for (int i = 0; i < 2048; ++i) { s = s * 1664525u + 1013904223u; hr[i] = ((s >> 8) / 16777216.f - 0.5f) * (i < 1024 ? 8.f : 100.f); }
  hipMemcpy(r, hr, sizeof hr, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep)
    for (int k32 = 0; k32 < 2; ++k32) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (k32) loop_kernel<1><<<blocks, 256>>>(out, cyc, iters, 1.7f);
      else loop_kernel<0><<<blocks, 256>>>(out, cyc, iters, 1.7f);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      long long hc[blocks]; hipMemcpy(hc, cyc, sizeof hc, hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < blocks; ++i) avg += hc[i]; avg /= blocks;
      printf("{\"mfma\": \"16x16x%d_bf16\", \"cycles_per_mfma\": %.2f, \"ms\": %.3f}\n", k32 ? 32 : 16, avg / (4.0 * iters), ms);
    }
  hipMemset(bad, 0, 4);
  eq_kernel<<<1, 64>>>(r, bad);
  int hb; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("{\"k16_vs_k32_zero_high_half_mismatches\": %d}\n", hb);
  return 0;
}
