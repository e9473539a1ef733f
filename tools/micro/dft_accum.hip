// Microbenchmark of the DFT accumulation: dft[p][f] += sum_u fr[u][p] *
// ph[u][f] (complex phase, real sample) for npts points, nfreq frequencies, n buffered updates,
// the product's wave-blocked layout [p/64][f][p%64] (complex).  Variants:
//   0  phases staged in LDS per 8-frequency tile (the product kernel of this round)
//   1  phases through wave-uniform (scalar) loads, 8-frequency tiles
//   2  phases in LDS, 16 points per lane group: a lane holds one point and 4 frequencies of a
//      16-frequency tile (lanes 0-15 / 16-31 / ... split the tile), samples from LDS
// Prints ms per call and the effective HBM rate of the algorithmic bytes.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/dft_accum.hip -o tools/micro/bin/dft_accum
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int KB = 32, FT = 8;

template <int W>
__device__ __forceinline__ void tile_lds(double2 *dp, const double2 *sph, const double *frv, int n,
                                         int i0, int woff) {
  double2 v[W];
#pragma unroll
  for (int w = 0; w < W; w++) v[w] = dp[(i0 + woff + w) * 64];
#pragma unroll
  for (int u = 0; u < KB; u++)
    if (u < n) {
#pragma unroll
      for (int w = 0; w < W; w++) {
        const double2 q = sph[u * FT + woff + w];
        v[w].x = v[w].x + frv[u] * q.x;
        v[w].y = v[w].y + frv[u] * q.y;
      }
    }
#pragma unroll
  for (int w = 0; w < W; w++) dp[(i0 + woff + w) * 64] = v[w];
}

__global__ __launch_bounds__(256) void acc_lds(double2 *dft, const double *fr, int n,
                                               const double2 *ph, int nfreq, long long npts) {
  __shared__ double2 sph[KB * FT];
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  const bool live = p < npts;
  double frv[KB];
#pragma unroll
  for (int u = 0; u < KB; u++) frv[u] = (live && u < n) ? fr[u * npts + p] : 0.0;
  double2 *dp = dft + (p >> 6) * nfreq * 64 + (p & 63);
  for (int i0 = 0; i0 < nfreq; i0 += FT) {
    const int ft = min(FT, nfreq - i0);
    __syncthreads();
    for (int e = threadIdx.x; e < n * FT; e += 256) {
      const int u = e / FT, w = e % FT;
      if (w < ft) sph[e] = ph[u * nfreq + i0 + w];
    }
    __syncthreads();
    if (!live) continue;
    if (ft == FT) {
      tile_lds<FT>(dp, sph, frv, n, i0, 0);
    } else {
      int w0 = 0;
      if (ft - w0 >= 4) tile_lds<4>(dp, sph, frv, n, i0, w0), w0 += 4;
      if (ft - w0 >= 2) tile_lds<2>(dp, sph, frv, n, i0, w0), w0 += 2;
      if (ft - w0 >= 1) tile_lds<1>(dp, sph, frv, n, i0, w0);
    }
  }
}

template <int W>
__device__ __forceinline__ void tile_s(double2 *dp, const double2 *php, const double *frv, int n,
                                       int i0) {
  double2 v[W];
#pragma unroll
  for (int w = 0; w < W; w++) v[w] = dp[(i0 + w) * 64];
#pragma unroll
  for (int u = 0; u < KB; u++)
    if (u < n) {
#pragma unroll
      for (int w = 0; w < W; w++) {
        const double2 q = php[u * 64 + i0 + w];  // uniform address: scalar loads
        v[w].x = v[w].x + frv[u] * q.x;
        v[w].y = v[w].y + frv[u] * q.y;
      }
    }
#pragma unroll
  for (int w = 0; w < W; w++) dp[(i0 + w) * 64] = v[w];
}

// phases [u][64] (padded rows) for uniform scalar addressing
__global__ __launch_bounds__(256) void acc_scalar(double2 *dft, const double *fr, int n,
                                                  const double2 *__restrict__ php, int nfreq,
                                                  long long npts) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npts) return;
  double frv[KB];
#pragma unroll
  for (int u = 0; u < KB; u++) frv[u] = u < n ? fr[u * npts + p] : 0.0;
  double2 *dp = dft + (p >> 6) * nfreq * 64 + (p & 63);
  int i0 = 0;
  for (; i0 + FT <= nfreq; i0 += FT) tile_s<FT>(dp, php, frv, n, i0);
  if (nfreq - i0 >= 4) tile_s<4>(dp, php, frv, n, i0), i0 += 4;
  if (nfreq - i0 >= 2) tile_s<2>(dp, php, frv, n, i0), i0 += 2;
  if (nfreq - i0 >= 1) tile_s<1>(dp, php, frv, n, i0);
}

int main(int argc, char **argv) {
  const long long npts = argc > 1 ? atoll(argv[1]) : 2000000;
  const int nfreq = argc > 2 ? atoi(argv[2]) : 50, n = argc > 3 ? atoi(argv[3]) : 32;
  const long long np = (npts + 63) & ~63LL;
  double2 *dft, *ph, *php;
  double *fr;
  hipMalloc(&dft, np * nfreq * sizeof(double2));
  hipMalloc(&fr, (size_t)KB * npts * 8);
  hipMalloc(&ph, (size_t)KB * nfreq * sizeof(double2));
  hipMalloc(&php, (size_t)KB * 64 * sizeof(double2));
  hipMemset(dft, 0, np * nfreq * sizeof(double2));
  hipMemset(fr, 0, (size_t)KB * npts * 8);
  hipMemset(ph, 0, (size_t)KB * nfreq * sizeof(double2));
  hipMemset(php, 0, (size_t)KB * 64 * sizeof(double2));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 2.0 * np * nfreq * 16 + (double)n * npts * 8;
  for (int var = 0; var < 2; var++) {
    float best = 1e9;
    for (int r = 0; r < 6; r++) {
      hipEventRecord(a);
      if (var == 0)
        acc_lds<<<(npts + 255) / 256, 256>>>(dft, fr, n, ph, nfreq, npts);
      else
        acc_scalar<<<(npts + 255) / 256, 256>>>(dft, fr, n, php, nfreq, npts);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r) best = ms < best ? ms : best;
    }
    printf("variant %d: npts %lld nfreq %d n %d: %.4f ms, %.0f GB/s (algorithmic)\n", var, npts,
           nfreq, n, best, bytes / (best * 1e-3) / 1e9);
  }
  return 0;
}
