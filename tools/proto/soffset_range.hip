// Probe (round 4): does a raw buffer load's range check include the scalar offset (soffset)?
// A 2 KB buffer of 1.0f, a descriptor over its first 1 KB; loads at (voffset, soffset) pairs
// past 1 KB print 0 if the range check covers that offset, 1 if it does not.
// hipcc -O3 --offload-arch=gfx950 tools/proto/soffset_range.hip -o tools/proto/soffset_range.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(const float* buf, float* out) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(buf), (short)0, 1024, 0x00020000);
  if (threadIdx.x == 0) {
    out[0] = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0);      // in range
    out[1] = __builtin_amdgcn_raw_buffer_load_b32(r, 1536, 0, 0);   // voffset past range
    out[2] = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 1536, 0);   // soffset past range
    out[3] = __builtin_amdgcn_raw_buffer_load_b32(r, 512, 1024, 0); // voffset in, sum past
  }
}

int main() {
  float *buf, *out;
  hipMalloc(&buf, 2048);
  hipMalloc(&out, 16);
  float h[512];
  for (int i = 0; i < 512; ++i) h[i] = 1.0f;
  hipMemcpy(buf, h, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, out);
  float o[4];
  hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
  std::printf("in-range %g  voffset-past %g  soffset-past %g  v-in+s-past %g\n", o[0], o[1], o[2], o[3]);
  return 0;
}
