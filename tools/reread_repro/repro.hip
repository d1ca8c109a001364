// Reduced reproduction of the round-3/4 finalize re-read mismatch (DESIGN
// §3): a wave-tile finalize that re-reads each candidate row from memory and
// keeps the best (score, value, index) with the round-3 branchy numpy-argmax
// comparison.  No uninitialised value is read on any path: every variable is
// written before use, better() is a pure function of its arguments.
//
//   hipcc --offload-arch=gfx950 -O3 repro.hip -o repro      (host + device)
//   hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only repro.hip -o repro.s
//   hipcc --offload-arch=gfx950 -O3 -S -emit-llvm --cuda-device-only repro.hip -o repro.ll
//   ./repro      -> "winners whose value is not their candidate's: N of M"
//
// -DSELECTS builds the shipped form (branch-free better() and selects).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#ifndef SELECTS
__device__ __forceinline__ bool better(double sa, int64_t ia, double sb, int64_t ib) {
  if (ia < 0) return false;
  if (ib < 0) return true;
  const bool na = sa != sa, nb = sb != sb;
  if (na || nb) return (na && nb) ? ia < ib : na;
  if (sa != sb) return sa > sb;
  return ia < ib;
}
#else
__device__ __forceinline__ bool better(double sa, int64_t ia, double sb, int64_t ib) {
  const bool na = sa != sa, nb = sb != sb;
  const bool lt = ia < ib;
  const bool by_score = (sa != sb) ? (sa > sb) : lt;
  const bool by_nan = (na && nb) ? lt : na;
  return (ia >= 0) & ((ib < 0) | ((na | nb) ? by_nan : by_score));
}
#endif

constexpr int KR = 2;

// score of a candidate: any function of the value that the compiler cannot
// fold (the production kernel's log-sum-exp EI plays this role)
__device__ __forceinline__ double score_of(double x, double c) { return -(x - c) * (x - c) + log(1.0 + x * x); }

__global__ __launch_bounds__(256) void k_finalize(const double *__restrict__ cand, int64_t n,
                                                  double c, double *out_s, double *out_v,
                                                  int64_t *out_i) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = ((int64_t)blockIdx.x * 4 + wave) * 64 * KR;
  int64_t li[KR];
  bool valid[KR];
  double x[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    li[r] = base + r * 64 + lane;
    valid[r] = li[r] < n;
    x[r] = valid[r] ? cand[li[r]] : 0.0;
  }
  double sc_reg[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) sc_reg[r] = score_of(x[r], c);
  double best_s = NAN, best_v = NAN;
  int64_t best_i = -1;
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    if (!valid[r]) continue;
    x[r] = cand[li[r]];  // the finalize re-read of the scored candidate
    // (LGMM: the lpdf subtracts log x of the re-read value, tpe.py:278-281)
    const double sc = sc_reg[r] - log(x[r]);
    const int64_t gi = li[r];
#ifndef SELECTS
    if (better(sc, gi, best_s, best_i)) {
      best_s = sc;
      best_v = x[r];
      best_i = gi;
    }
#else
    const bool b = better(sc, gi, best_s, best_i);
    best_s = b ? sc : best_s;
    best_v = b ? x[r] : best_v;
    best_i = b ? gi : best_i;
#endif
  }
  const int64_t t = ((int64_t)blockIdx.x * 4 + wave) * 64 + lane;
  out_s[t] = best_s;
  out_v[t] = best_v;
  out_i[t] = best_i;
}

int main() {
  const int64_t n = 1 << 22;
  const double c = 0.3;
  double *h = (double *)malloc(n * sizeof(double));
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (int64_t i = 0; i < n; ++i) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    h[i] = (double)(st >> 11) * 0x1.0p-53 * 2.0 - 1.0;
  }
  const int64_t lanes = n / KR;
  double *d, *os, *ov;
  int64_t *oi;
  hipMalloc(&d, n * sizeof(double));
  hipMalloc(&os, lanes * sizeof(double));
  hipMalloc(&ov, lanes * sizeof(double));
  hipMalloc(&oi, lanes * sizeof(int64_t));
  hipMemcpy(d, h, n * sizeof(double), hipMemcpyHostToDevice);
  k_finalize<<<(unsigned)(lanes / 256), 256>>>(d, n, c, os, ov, oi);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
  double *hv = (double *)malloc(lanes * sizeof(double));
  int64_t *hi = (int64_t *)malloc(lanes * sizeof(int64_t));
  hipMemcpy(hv, ov, lanes * sizeof(double), hipMemcpyDeviceToHost);
  hipMemcpy(hi, oi, lanes * sizeof(int64_t), hipMemcpyDeviceToHost);
  int64_t bad = 0, row1 = 0;
  for (int64_t t = 0; t < lanes; ++t) {
    const int64_t i = hi[t];
    if (i < 0 || i >= n) { ++bad; continue; }
    row1 += ((i / 64) % KR) == 1;
    if (hv[t] != h[i]) ++bad;
  }
  printf("winners whose value is not their candidate's: %lld of %lld (row-1 winners %lld)\n",
         (long long)bad, (long long)lanes, (long long)row1);
  return bad ? 1 : 0;
}
