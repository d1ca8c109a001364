// Instruction-fetch cost probe (diagnostic): the same 4 x 2048 dependent
// fp32 FMAs per thread, once as straight-line code (~64 KB, every line
// fetched for the first time in the launch) and once as a small unrolled loop
// (body stays in the instruction cache).  Prints wall-clock ns per FMA.
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool STRAIGHT>
__global__ __launch_bounds__(1024) void k(float *out, unsigned long long *t, float a, float b) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  if constexpr (STRAIGHT) {
#pragma unroll
    for (int i = 0; i < 2048; ++i) {
      x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
    }
  } else {
#pragma unroll 16
    for (int i = 0; i < 2048; ++i) {
      x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
    }
  }
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 1024 + threadIdx.x] = x0 + x1 + x2 + x3;
}

int main() {
  float *out;
  unsigned long long *t, h[64];
  hipMalloc(&out, 64 * 1024 * 4);
  hipMalloc(&t, 64 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 2; ++v) {
      for (int nb : {1, 40}) {
        if (v == 0) k<true><<<nb, 1024>>>(out, t, 0.999f, 0.001f);
        else k<false><<<nb, 1024>>>(out, t, 0.999f, 0.001f);
        hipMemcpy(h, t, nb * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < nb; ++i) s += h[i];
        s /= nb;
        printf("rep %d %s blocks %2d: %.2f us, %.2f ns per FMA instruction per wave\n", rep,
               v == 0 ? "straight-line" : "loop         ", nb, s / 100.0, s * 10.0 / (4 * 2048));
      }
    }
  }
  return 0;
}
