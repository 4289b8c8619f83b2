// Check that the crossbar-free wave reductions (common.hpp wave_sum / wave_max: permlane32 /
// permlane16 swaps + DPP row rotations) return the bits of the __shfl_xor butterfly they
// replace (xor 32, 16, 8, 4, 2, 1 in that order) on every lane.  Built by
// tools/wave_reduce_check.sh into tools/_ab/wave_reduce_check.so; run on the GPU with
// python tools/wave_reduce_check.py.
#include "common.hpp"

namespace {
__device__ float ref_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ float ref_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__global__ void check_kernel(const float* in, int n, unsigned* bad) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x * blockDim.x >= n) return;
  const float v = in[i < n ? i : n - 1];
  const float a = wave_sum(v), b = ref_sum(v);
  const float c = wave_max(v), d = ref_max(v);
  if (__float_as_uint(a) != __float_as_uint(b)) atomicAdd(bad, 1u);
  if (__float_as_uint(c) != __float_as_uint(d)) atomicAdd(bad + 1, 1u);
  // single xor partners, float and int, every o
  const int iv = __float_as_int(v) ^ (int)i;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    if (__float_as_uint(xor_lane(v, o)) != __float_as_uint(__shfl_xor(v, o, 64))) atomicAdd(bad + 2, 1u);
    if (xor_lane(iv, o) != __shfl_xor(iv, o, 64)) atomicAdd(bad + 2, 1u);
  }
  // an ascending butterfly (o = 4, 8, 16, 32: the decode heads' partial-sum merge)
  float e = v, f = v;
#pragma unroll
  for (int o = 4; o < 64; o <<= 1) {
    e += xor_lane(e, o);
    f += __shfl_xor(f, o, 64);
  }
  if (__float_as_uint(e) != __float_as_uint(f)) atomicAdd(bad + 3, 1u);
}
}  // namespace

extern "C" int wave_reduce_check(const float* in, int n, unsigned* bad) {
  hipLaunchKernelGGL(check_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, in, n, bad);
  return hipDeviceSynchronize() != hipSuccess;
}
