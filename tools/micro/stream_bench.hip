// Microbenchmark: achievable HBM bandwidth for the fused step's access
// pattern (9 streamed reads + 6 streamed writes of f64 per cell) under
// different traversal orders and layouts.  Not part of the product; it guides
// the kernel design (DESIGN.md "Measured access-pattern ceilings").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

struct Arr { const double *r[9]; double *w[6]; };
constexpr int NX = 528, NY = 528, NZ = 520;
constexpr long long ST1 = NX, ST2 = (long long)NX * NY, NT = ST2 * NZ;

template <int NR, int NW>
__global__ void k_lin(Arr a, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    double s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < NR; c++) s[c] = a.r[c][i];
    double acc = 0;
#pragma unroll
    for (int c = 0; c < 9; c++) acc += s[c];
#pragma unroll
    for (int c = 0; c < NW; c++) a.w[c][i] = acc * (c + 1);
    if (NW == 0 && acc == 12345.0) a.w[0][i] = acc;
  }
}

// AoS: 3 fields (Bo, Do, u) of 3 comps read, 2 fields (Bn, Dn) written; 24 B per field-cell
__global__ void k_lin_aos(Arr a, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    double s[9];
#pragma unroll
    for (int f = 0; f < 3; f++)
#pragma unroll
      for (int c = 0; c < 3; c++) s[3 * f + c] = a.r[f][3 * i + c];
#pragma unroll
    for (int f = 0; f < 2; f++)
#pragma unroll
      for (int c = 0; c < 3; c++) a.w[f][3 * i + c] = s[c + 3 * f] * s[6 + c];
  }
}

// one block per (x,y) tile of 64 x FYB columns, z march over zc planes
template <int FYB>
__global__ void k_march(Arr a, int zc) {
  const int gx = 8 + blockIdx.x * 64 + threadIdx.x, gy = 8 + blockIdx.y * FYB + threadIdx.y;
  const int z0 = 4 + blockIdx.z * zc;
  const unsigned cb = (unsigned)((gx + gy * ST1) * 8);
  for (int k = z0; k < z0 + zc; k++) {
    const unsigned o = cb + (unsigned)k * (unsigned)(ST2 * 8);
    double s[9];
#pragma unroll
    for (int c = 0; c < 9; c++) s[c] = *(const double *)((const char *)a.r[c] + o);
#pragma unroll
    for (int c = 0; c < 6; c++) *(double *)((char *)a.w[c] + o) = s[c] * s[c + 3] + s[(c + 6) % 9];
  }
}


// software-pipelined march: loads for plane k+DIST issued before the stores of plane k
template <int FYB, int DIST>
__global__ void k_march_pipe(Arr a, int zc) {
  const int gx = 8 + blockIdx.x * 64 + threadIdx.x, gy = 8 + blockIdx.y * FYB + threadIdx.y;
  const int z0 = 4 + blockIdx.z * zc, z1 = z0 + zc;
  const unsigned cb = (unsigned)((gx + gy * ST1) * 8);
  const unsigned s2 = (unsigned)(ST2 * 8);
  double q[DIST + 1][9];
  auto ld = [&](double *d, int k) {
    const unsigned o = cb + (unsigned)min(k, z1 - 1) * s2;
#pragma unroll
    for (int c = 0; c < 9; c++) d[c] = *(const double *)((const char *)a.r[c] + o);
  };
#pragma unroll
  for (int j = 0; j < DIST; j++) ld(q[j], z0 + j);
  for (int k = z0; k < z1; k += DIST + 1) {
#pragma unroll
    for (int j = 0; j <= DIST; j++) {
      const int kk = k + j;
      ld(q[(j + DIST) % (DIST + 1)], kk + DIST);
      const double *s = q[j];
      if (kk < z1) {
        const unsigned o = cb + (unsigned)kk * s2;
#pragma unroll
        for (int c = 0; c < 6; c++) *(double *)((char *)a.w[c] + o) = s[c] * s[c + 3] + s[(c + 6) % 9];
      }
    }
  }
}


// wide march: block covers WX contiguous x cells (one per thread) x FYB rows
template <int WX, int FYB>
__global__ void k_march_wide(Arr a, int zc) {
  const int gx = 16 + threadIdx.x, gy = 8 + blockIdx.x * FYB + threadIdx.y;
  const int z0 = 4 + blockIdx.y * zc;
  const unsigned cb = (unsigned)((gx + gy * ST1) * 8);
  for (int k = z0; k < z0 + zc; k++) {
    const unsigned o = cb + (unsigned)k * (unsigned)(ST2 * 8);
    double s[9];
#pragma unroll
    for (int c = 0; c < 9; c++) s[c] = *(const double *)((const char *)a.r[c] + o);
#pragma unroll
    for (int c = 0; c < 6; c++) *(double *)((char *)a.w[c] + o) = s[c] * s[c + 3] + s[(c + 6) % 9];
  }
}
// tiled layout: each (tile, plane) chunk of 64x16 doubles is contiguous
__global__ void k_march_tiled(Arr a, int zc) {
  const int tile = blockIdx.x + blockIdx.y * 8;  // 8 x 32 tiles
  const int z0 = blockIdx.z * zc;
  const unsigned lane = threadIdx.x + threadIdx.y * 64;
  for (int k = z0; k < z0 + zc; k++) {
    const unsigned o = (unsigned)(((k * 256 + tile) * 1024 + lane) * 8);
    double s[9];
#pragma unroll
    for (int c = 0; c < 9; c++) s[c] = *(const double *)((const char *)a.r[c] + o);
#pragma unroll
    for (int c = 0; c < 6; c++) *(double *)((char *)a.w[c] + o) = s[c] * s[c + 3] + s[(c + 6) % 9];
  }
}
// aligned 64x16 march (x starts on a 128-B boundary)
__global__ void k_march_al(Arr a, int zc) {
  const int gx = 16 + blockIdx.x * 64 + threadIdx.x, gy = 8 + blockIdx.y * 16 + threadIdx.y;
  const int z0 = 4 + blockIdx.z * zc;
  const unsigned cb = (unsigned)((gx + gy * ST1) * 8);
  for (int k = z0; k < z0 + zc; k++) {
    const unsigned o = cb + (unsigned)k * (unsigned)(ST2 * 8);
    double s[9];
#pragma unroll
    for (int c = 0; c < 9; c++) s[c] = *(const double *)((const char *)a.r[c] + o);
#pragma unroll
    for (int c = 0; c < 6; c++) *(double *)((char *)a.w[c] + o) = s[c] * s[c + 3] + s[(c + 6) % 9];
  }
}

// full-row blocks: block of 512 threads covers one full x row; grid (y, z)
__global__ void k_rows(Arr a) {
  const int gx = 8 + threadIdx.x, gy = 8 + blockIdx.x, gz = 4 + blockIdx.y;
  const long long o = gx + gy * ST1 + gz * ST2;
  double s[9];
#pragma unroll
  for (int c = 0; c < 9; c++) s[c] = a.r[c][o];
#pragma unroll
  for (int c = 0; c < 6; c++) a.w[c][o] = s[c] * s[c + 3] + s[(c + 6) % 9];
}

int main() {
  std::vector<double *> bufs(15);
  for (int i = 0; i < 15; i++) { CK(hipMalloc(&bufs[i], NT * 8)); CK(hipMemset(bufs[i], 0, NT * 8)); }
  Arr a;
  for (int i = 0; i < 9; i++) a.r[i] = bufs[i];
  for (int i = 0; i < 6; i++) a.w[i] = bufs[9 + i];
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char *name, auto launch, double bytes) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; r++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const double N = 512.0 * 512 * 512;
  const long long n = 512LL * 512 * 512;
  run("lin 1R1W", [&] { k_lin<1, 1><<<256 * 64, 256>>>(a, n); }, N * 16);
  run("lin 2R1W", [&] { k_lin<2, 1><<<256 * 64, 256>>>(a, n); }, N * 24);
  run("lin 9R0W", [&] { k_lin<9, 0><<<256 * 64, 256>>>(a, n); }, N * 72);
  run("lin 0R6W", [&] { k_lin<0, 6><<<256 * 64, 256>>>(a, n); }, N * 48);
  run("lin 9R6W", [&] { k_lin<9, 6><<<256 * 64, 256>>>(a, n); }, N * 120);
  run("lin 9R6W grid 256x8", [&] { k_lin<9, 6><<<256 * 8, 256>>>(a, n); }, N * 120);
  run("lin 9R6W grid 256x512", [&] { k_lin<9, 6><<<256 * 512, 256>>>(a, n); }, N * 120);
  run("lin AoS 3R2W (x3 comps)", [&] { k_lin_aos<<<256 * 64, 256>>>(a, n / 3); }, N / 3 * 120);
  run("rows 512 (grid y,z)", [&] { k_rows<<<dim3(512, 512), 512>>>(a); }, N * 120);
  for (int zc : {1, 64, 512}) {
    char nm[64];
    snprintf(nm, 64, "wide 512x1 zc=%d", zc);
    run(nm, [&] { k_march_wide<512, 1><<<dim3(512, 512 / zc), dim3(512, 1)>>>(a, zc); }, N * 120);
    snprintf(nm, 64, "wide 512x2 zc=%d", zc);
    run(nm, [&] { k_march_wide<512, 2><<<dim3(256, 512 / zc), dim3(512, 2)>>>(a, zc); }, N * 120);
    snprintf(nm, 64, "wide 256x4 zc=%d", zc);
    run(nm, [&] { k_march_wide<256, 4><<<dim3(128, 512 / zc), dim3(256, 4)>>>(a, zc); }, N * 120);
    snprintf(nm, 64, "tiled 64x16 zc=%d", zc);
    run(nm, [&] { k_march_tiled<<<dim3(8, 32, 512 / zc), dim3(64, 16)>>>(a, zc); }, N * 120);
    snprintf(nm, 64, "aligned 64x16 zc=%d", zc);
    run(nm, [&] { k_march_al<<<dim3(8, 32, 512 / zc), dim3(64, 16)>>>(a, zc); }, N * 120);
    snprintf(nm, 64, "march 64x16 zc=%d", zc);
    run(nm, [&] { k_march<16><<<dim3(8, 32, 512 / zc), dim3(64, 16)>>>(a, zc); }, N * 120);
  }
  return 0;
}
