// Latency probes for k_fit design (diagnostic only): cycles per s_barrier
// with 16 / 4 waves, per dependent LDS load, per dependent __shfl_xor, per
// dependent global load (L2 hit).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(long long *out, int iters, const int *gbuf) {
  __shared__ int lds[1024];
  const int t = threadIdx.x;
  lds[t & 1023] = (t + 1) & 1023;
  __syncthreads();
  long long c0 = clock64();
  for (int i = 0; i < iters; ++i) __syncthreads();
  long long c1 = clock64();
  int p = t & 1023;
  for (int i = 0; i < iters; ++i) p = lds[p];
  long long c2 = clock64();
  int v = t;
  for (int i = 0; i < iters; ++i) v = __shfl_xor(v, 16, 64) + 1;
  long long c3 = clock64();
  int q = t & 1023;
  for (int i = 0; i < iters; ++i) q = gbuf[q];
  long long c4 = clock64();
  int u = t;
  for (int i = 0; i < iters; ++i) u = __shfl_xor(u, 1, 64) + 1;
  long long c5 = clock64();
  if (t == 0) {
    out[0] = (c1 - c0) / iters;
    out[1] = (c2 - c1) / iters;
    out[2] = (c3 - c2) / iters;
    out[3] = (c4 - c3) / iters;
    out[4] = (c5 - c4) / iters;
    out[5] = p + v + q + u;
  }
}

int main() {
  long long *d, h[6];
  int *g;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&g, 4096 * 4);
  int hg[4096];
  for (int i = 0; i < 4096; ++i) hg[i] = (i * 97 + 13) & 1023;
  hipMemcpy(g, hg, sizeof(hg), hipMemcpyHostToDevice);
  for (int threads : {1024, 256, 64}) {
    for (int rep = 0; rep < 2; ++rep) {
      k_lat<<<1, threads>>>(d, 256, g);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    }
    printf("threads %4d: barrier %lld  lds-chain %lld  shfl16-chain %lld  global-chain %lld  shfl1-chain %lld cycles\n",
           threads, h[0], h[1], h[2], h[3], h[4]);
  }
  return 0;
}
