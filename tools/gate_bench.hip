// Microbenchmark of the update pass's per-hit-point recurrence (gate_round in
// ceng795_amd/csrc/ppm_kernels.hip) on synthetic rounds, one wave per workgroup.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
//         -I ceng795_amd/csrc tools/gate_bench.hip -o build/gate_bench
//   build/gate_bench [n=341] [blocks=1] [reps=200] [dmax=0.9]
// Prints core-clock cycles per candidate of (R)+(K) and of the whole round (diag ticks are
// 100 MHz; clock64 here is the shader clock).  Development tool; not part of the product.
#include "ppm_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace ppm {
namespace {
constexpr int kGateKMaxBench = 64 * kGateK;
__global__ __launch_bounds__(64) void gate_bench_kernel(int n, int reps, const float* rr_table,
                                                         int nrr, float dmax, float* out,
                                                         unsigned long long* ticks) {
  __shared__ float4 rec[kGateKMaxBench + 4];
  __shared__ float4 acc[kGateKMaxBench + 4];
  __shared__ float rrb[2 * kGateKMaxBench + 8];
  __shared__ float R[kGateKMaxBench + 9];
  __shared__ float d2s[kGateKMaxBench];
  const int lane = (int)__lane_id();
  for (int i = lane; i < 2 * kGateKMaxBench + 8; i += 64) rrb[i] = rr_table[1000 + i];
  // distances: ~90 % accepted (R shrinks from 1 by the rr products)
  unsigned s = 12345u + 77u * blockIdx.x;
  for (int k = lane; k < n; k += 64) {
    s = s * 1664525u + 1013904223u + (unsigned)k * 2654435761u;
    d2s[k] = (float)(s >> 8) * (1.0f / 16777216.0f) * dmax;
  }
  __syncthreads();
  float fx = 0, fy = 0, fz = 0, r2 = 1.0f;
  unsigned cnt = 1000;
  unsigned long long t[2] = {0, 0};
  unsigned long long c0 = 0, cyc = 0;
  for (int r = 0; r < reps; r++) {
    for (int k = lane; k < n; k += 64) rec[k] = make_float4(0.5f, 0.25f, 0.125f, d2s[k]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    r2 = 1.0f;
    c0 = clock64();
    gate_round(rec, acc, n, false, nullptr, rr_table, nrr, rrb, R, fx, fy, fz, r2, cnt, t);
    cyc += clock64() - c0;
    cnt = 1000;
  }
  if (lane == 0) {
    out[blockIdx.x] = fx + fy + fz + r2;
    ticks[3 * blockIdx.x] = cyc;
    ticks[3 * blockIdx.x + 1] = t[0];
    ticks[3 * blockIdx.x + 2] = t[1];
  }
}
}  // namespace
}  // namespace ppm

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 341;
  const int blocks = argc > 2 ? std::atoi(argv[2]) : 1;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 200;
  const float dmax = argc > 4 ? (float)std::atof(argv[4]) : 0.9f;  // d2 ~ U(0, dmax): 1.8 ~ half accepted
  if (n > ppm::kGateKMaxBench) return 2;
  const int nrr = 1 << 16;
  std::vector<float> rr(nrr);
  for (int i = 0; i < nrr; i++) {
    const float nf = (float)i * 0.7f;
    rr[i] = (float)((double)(nf + 0.7f) / ((double)nf + 1.0));
  }
  float *d_rr, *d_out;
  unsigned long long* d_t;
  hipMalloc(&d_rr, nrr * 4);
  hipMalloc(&d_out, blocks * 4);
  hipMalloc(&d_t, blocks * 24);
  hipMemcpy(d_rr, rr.data(), nrr * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(ppm::gate_bench_kernel, dim3(blocks), dim3(64), 0, 0, n, 2, d_rr, nrr, dmax, d_out, d_t);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(ppm::gate_bench_kernel, dim3(blocks), dim3(64), 0, 0, n, reps, d_rr, nrr, dmax, d_out, d_t);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> t(3 * blocks);
  hipMemcpy(t.data(), d_t, blocks * 24, hipMemcpyDeviceToHost);
  const double per = (double)reps * n;
  std::printf("{\"dmax\": %.2f, \"n\": %d, \"blocks\": %d, \"reps\": %d, \"kernel_ms\": %.3f, "
              "\"cycles_per_candidate\": %.1f, \"RK_ns_per_candidate\": %.1f, "
              "\"all_ns_per_candidate\": %.1f}\n",
              dmax, n, blocks, reps, ms, t[0] / per, t[1] * 10.0 / per, t[2] * 10.0 / per);
  return 0;
}
