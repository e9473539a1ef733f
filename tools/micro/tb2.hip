// Temporal-blocking prototype ("next"): two Yee steps per z-march
// against one, on the lean case (vacuum interior, E == D, H == B, cells outside
// [2, N-3]^3 held fixed), bit-exact against a naive one-point-per-thread step.
// Not part of the product: it measures what a 2-step tile kernel can reach on gfx950
// before the product's bodies (PML, palette, sources, DFT, ranks) are given 2-step forms.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tb2 tools/micro/tb2.hip
//   ./tb2 [N=512] [chunk=32] [reps=10]
//
// Work item = (tile, z chunk).  Lanes cover 64 x 16 points (x0-8 .. x0+55, y0-2 .. y0+13);
// step n -> n+1 runs on all of them, step n+1 -> n+2 is valid on lanes 2..61 / rows 2..13,
// of which the 48 x 12 own points (x0 .. x0+47: whole 64-B sectors) are stored.  The march
// runs step n at plane k and step n+1 at plane k-1; step n+1 takes E^{n+1}(k) and B^{n+1}(k-1)
// from registers, so per two steps each point's D, B are loaded once and stored once.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct Grid {
  int nx, ny, nz;
  double C;
};
struct F6 {
  double *d[3], *b[3];
};

// one component update each, the same expression (and operand order) in every kernel
__device__ __forceinline__ double bup(double b, double a_p, double a, double c_p, double c, double C) {
  return b - C * ((a_p - a) - (c_p - c));
}
__device__ __forceinline__ double dup(double d, double a, double a_m, double c, double c_m, double C) {
  return d + C * ((a - a_m) - (c - c_m));
}
__device__ __forceinline__ bool upd(const Grid &g, int i, int j, int k) {
  return i >= 2 && i <= g.nx - 3 && j >= 2 && j <= g.ny - 3 && k >= 2 && k <= g.nz - 3;
}
__device__ __forceinline__ long long at(const Grid &g, int i, int j, int k) {
  return (long long)i + (long long)g.nx * ((long long)j + (long long)g.ny * k);
}

// ---- naive reference: B step then D step, one point per thread, src -> dst
__global__ void ref_b(Grid g, F6 s, F6 t) {
  const long long n = (long long)g.nx * g.ny * g.nz;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < n;
       p += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(p % g.nx), j = (int)((p / g.nx) % g.ny), k = (int)(p / ((long long)g.nx * g.ny));
    if (!upd(g, i, j, k)) {
      for (int c = 0; c < 3; c++) t.b[c][p] = s.b[c][p];
      continue;
    }
    const long long px = p + 1, py = p + g.nx, pz = p + (long long)g.nx * g.ny;
    t.b[0][p] = bup(s.b[0][p], s.d[2][py], s.d[2][p], s.d[1][pz], s.d[1][p], g.C);
    t.b[1][p] = bup(s.b[1][p], s.d[0][pz], s.d[0][p], s.d[2][px], s.d[2][p], g.C);
    t.b[2][p] = bup(s.b[2][p], s.d[1][px], s.d[1][p], s.d[0][py], s.d[0][p], g.C);
  }
}
__global__ void ref_d(Grid g, F6 s, F6 t) {  // reads t.b (new B), s.d; writes t.d
  const long long n = (long long)g.nx * g.ny * g.nz;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < n;
       p += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(p % g.nx), j = (int)((p / g.nx) % g.ny), k = (int)(p / ((long long)g.nx * g.ny));
    if (!upd(g, i, j, k)) {
      for (int c = 0; c < 3; c++) t.d[c][p] = s.d[c][p];
      continue;
    }
    const long long mx = p - 1, my = p - g.nx, mz = p - (long long)g.nx * g.ny;
    t.d[0][p] = dup(s.d[0][p], t.b[2][p], t.b[2][my], t.b[1][p], t.b[1][mz], g.C);
    t.d[1][p] = dup(s.d[1][p], t.b[0][p], t.b[0][mz], t.b[2][p], t.b[2][mx], g.C);
    t.d[2][p] = dup(s.d[2][p], t.b[1][p], t.b[1][mx], t.b[0][p], t.b[0][my], g.C);
  }
}

// ---- tile kernels: TWO = 2-step march, else the same structure doing one step
constexpr int LX = 64, LY = 16, HYL = 2, OWNY = 12;
// x shape: own columns per tile OX, lanes left of them HX, origin X0 of tile 0's own
// range (48 / 8 / -40: 512-B aligned loads, whole-sector stores; 56 / 4 / -52: 64-B aligned
// loads, 32-B offset stores, 17 % more own points per item)

template <bool TWO, bool PF = false, int OWNX = 48, int HXL = 8, int X0 = -40>  // PF: prefetch
__global__ __launch_bounds__(1024) void tile_kernel(Grid g, F6 s, F6 t, int ntx, int nty, int chunk) {
  __shared__ double sE1[3][LY][LX], sH1[3][LY][LX], sE2[3][LY][LX], sH2[3][LY][LX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int item = blockIdx.x;
  const int tx = item % ntx;
  item /= ntx;
  const int ty = item % nty;
  const int ch = item / nty;
  const int x0 = X0 + OWNX * tx, y0 = 2 + OWNY * ty;
  const int zs = 2 + chunk * ch, ze = min(zs + chunk, g.nz - 2);
  const int i = x0 - HXL + lane, j = y0 - HYL + w;
  const int ic = min(max(i, 0), g.nx - 1), jc = min(max(j, 0), g.ny - 1);
  const bool own = lane >= HXL && lane < HXL + OWNX && w >= HYL && w < HYL + OWNY && i < g.nx && j < g.ny;
  const int lp = min(lane + 1, LX - 1), lm = max(lane - 1, 0), wp = min(w + 1, LY - 1), wm = max(w - 1, 0);
  const long long plane = (long long)g.nx * g.ny;
  const long long col = (long long)ic + (long long)g.nx * jc;
  auto zc = [&](int k) { return min(max(k, 0), g.nz - 1); };
  const double C = g.C;
  const int k0 = TWO ? zs - 2 : zs - 1;
  // E^n(k0) (== D), then the march
  double en0, en1, en2;
  {
    const long long o = col + plane * zc(k0);
    en0 = s.d[0][o], en1 = s.d[1][o], en2 = s.d[2][o];
  }
  double h1x = 0, h1y = 0;                 // B^{n+1}(k-1) x, y (z-derivative of curl H)
  double b1m0 = 0, b1m1 = 0, b1m2 = 0;     // B^{n+1}(k-1)
  double d1m0 = 0, d1m1 = 0, d1m2 = 0;     // D^{n+1}(k-1) == E^{n+1}(k-1)
  double h2x = 0, h2y = 0;                 // B^{n+2}(j-1) x, y
  double pe0 = 0, pe1 = 0, pe2 = 0, pb0 = 0, pb1 = 0, pb2 = 0;
  if (PF) {
    const long long o = col + plane * zc(k0), o1 = col + plane * zc(k0 + 1);
    pe0 = s.d[0][o1], pe1 = s.d[1][o1], pe2 = s.d[2][o1];
    pb0 = s.b[0][o], pb1 = s.b[1][o], pb2 = s.b[2][o];
  }
  for (int k = k0; k <= (TWO ? ze : ze - 1); k++) {
    const long long o = col + plane * zc(k), o1 = col + plane * zc(k + 1);
    double e10, e11, e12, bn0, bn1, bn2;  // E^n(k+1), B^n(k)
    if (PF) {
      e10 = pe0, e11 = pe1, e12 = pe2, bn0 = pb0, bn1 = pb1, bn2 = pb2;
      const long long o2 = col + plane * zc(k + 2);
      pe0 = s.d[0][o2], pe1 = s.d[1][o2], pe2 = s.d[2][o2];
      pb0 = s.b[0][o1], pb1 = s.b[1][o1], pb2 = s.b[2][o1];
    } else {
      e10 = s.d[0][o1], e11 = s.d[1][o1], e12 = s.d[2][o1];
      bn0 = s.b[0][o], bn1 = s.b[1][o], bn2 = s.b[2][o];
    }
    sE1[0][w][lane] = en0, sE1[1][w][lane] = en1, sE1[2][w][lane] = en2;
    if (TWO) sE2[0][w][lane] = d1m0, sE2[1][w][lane] = d1m1, sE2[2][w][lane] = d1m2;
    __syncthreads();  // A
    const bool u1 = upd(g, i, j, k);
    double b10 = bn0, b11 = bn1, b12 = bn2;
    if (u1) {
      b10 = bup(bn0, sE1[2][wp][lane], en2, e11, en1, C);
      b11 = bup(bn1, e10, en0, sE1[2][w][lp], en2, C);
      b12 = bup(bn2, sE1[1][w][lp], en1, sE1[0][wp][lane], en0, C);
    }
    sH1[0][w][lane] = b10, sH1[1][w][lane] = b11, sH1[2][w][lane] = b12;
    __syncthreads();  // B
    double d10 = en0, d11 = en1, d12 = en2;
    if (u1) {
      d10 = dup(en0, b12, sH1[2][wm][lane], b11, h1y, C);
      d11 = dup(en1, b10, h1x, b12, sH1[2][w][lm], C);
      d12 = dup(en2, b11, sH1[1][w][lm], b10, sH1[0][wm][lane], C);
    }
    if (!TWO) {
      if (own && k >= zs && k < ze && u1) {
        t.b[0][o] = b10, t.b[1][o] = b11, t.b[2][o] = b12;
        t.d[0][o] = d10, t.d[1][o] = d11, t.d[2][o] = d12;
      }
    } else {
      // step n+1 at plane jz = k - 1: E^{n+1}(jz) = d1m (in sE2), E^{n+1}(jz+1) = d1 (own)
      const int jz = k - 1;
      const bool u2 = upd(g, i, j, jz);
      double b20 = b1m0, b21 = b1m1, b22 = b1m2;
      if (u2) {
        b20 = bup(b1m0, sE2[2][wp][lane], d1m2, d11, d1m1, C);
        b21 = bup(b1m1, d10, d1m0, sE2[2][w][lp], d1m2, C);
        b22 = bup(b1m2, sE2[1][w][lp], d1m1, sE2[0][wp][lane], d1m0, C);
      }
      sH2[0][w][lane] = b20, sH2[1][w][lane] = b21, sH2[2][w][lane] = b22;
      __syncthreads();  // C
      double d20 = d1m0, d21 = d1m1, d22 = d1m2;
      if (u2) {
        d20 = dup(d1m0, b22, sH2[2][wm][lane], b21, h2y, C);
        d21 = dup(d1m1, b20, h2x, b22, sH2[2][w][lm], C);
        d22 = dup(d1m2, b21, sH2[1][w][lm], b20, sH2[0][wm][lane], C);
      }
      if (own && jz >= zs && jz < ze && u2) {
        const long long oj = col + plane * jz;
        t.b[0][oj] = b20, t.b[1][oj] = b21, t.b[2][oj] = b22;
        t.d[0][oj] = d20, t.d[1][oj] = d21, t.d[2][oj] = d22;
      }
      h2x = b20, h2y = b21;
      b1m0 = b10, b1m1 = b11, b1m2 = b12;
      d1m0 = d10, d1m1 = d11, d1m2 = d12;
    }
    h1x = b10, h1y = b11;
    en0 = e10, en1 = e11, en2 = e12;
    if (!TWO) __syncthreads();  // sE1 / sH1 reads done before the next plane's writes
  }
}

__global__ void init_kernel(double *p, long long n, unsigned seed) {
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    unsigned long long x = (unsigned long long)q * 0x9E3779B97F4A7C15ULL + seed;
    x ^= x >> 31, x *= 0xBF58476D1CE4E5B9ULL, x ^= x >> 29;
    p[q] = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

static F6 alloc6(long long n) {
  F6 f;
  for (int c = 0; c < 3; c++) {
    CK(hipMalloc(&f.d[c], n * 8));
    CK(hipMalloc(&f.b[c], n * 8));
  }
  return f;
}
static void copy6(F6 dst, F6 src, long long n) {
  for (int c = 0; c < 3; c++) {
    CK(hipMemcpy(dst.d[c], src.d[c], n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(dst.b[c], src.b[c], n * 8, hipMemcpyDeviceToDevice));
  }
}
static bool same6(F6 a, F6 b, long long n, const char *what) {
  std::vector<double> x(n), y(n);
  bool ok = true;
  for (int c = 0; c < 6; c++) {
    CK(hipMemcpy(x.data(), c < 3 ? a.d[c] : a.b[c - 3], n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), c < 3 ? b.d[c] : b.b[c - 3], n * 8, hipMemcpyDeviceToHost));
    long long bad = 0;
    for (long long q = 0; q < n; q++) bad += memcmp(&x[q], &y[q], 8) != 0;
    if (bad) printf("%s: component %d differs at %lld points\n", what, c, bad), ok = false;
  }
  return ok;
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 512;
  const int chunk = argc > 2 ? atoi(argv[2]) : 32;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  Grid g{N, N, N, 0.5};
  const long long n = (long long)N * N * N;
  F6 A = alloc6(n), B = alloc6(n), R = alloc6(n), S = alloc6(n);
  for (int c = 0; c < 3; c++) {
    init_kernel<<<4096, 256>>>(A.d[c], n, 11 + c);
    init_kernel<<<4096, 256>>>(A.b[c], n, 101 + c);
  }
  CK(hipDeviceSynchronize());
  const int OWNX = 48;
  const int ntx = (N - 3 + 40) / OWNX + 1, nty = (N - 5) / OWNY + 1, nch = (N - 4 + chunk - 1) / chunk;
  const int ntx56 = (N - 3 + 52) / 56 + 1, items56 = ntx56 * nty * nch;
  const int items = ntx * nty * nch;
  // shapes the kernels assume (checked before any launch)
  if (N < 16 || chunk < 1 || -40 + OWNX * (ntx - 1) > N - 3 || 2 + OWNY * (nty - 1) > N - 3 ||
      -40 + OWNX * ntx <= N - 3 || 2 + OWNY * nty <= N - 3) {
    fprintf(stderr, "bad shape\n");
    return 1;
  }
  // parity: naive 2 steps vs one 2-step launch vs two 1-step tile launches
  copy6(R, A, n);
  copy6(S, A, n);
  for (int st = 0; st < 2; st++) {
    ref_b<<<8192, 256>>>(g, R, S);
    ref_d<<<8192, 256>>>(g, R, S);
    copy6(R, S, n);  // R = the state after this step
  }
  copy6(B, A, n);  // the tile kernels store only updated own points: boundaries come from the copy
  tile_kernel<true><<<items, 1024>>>(g, A, B, ntx, nty, chunk);
  CK(hipDeviceSynchronize());
  bool ok2 = same6(B, R, n, "2-step tile vs naive");
  copy6(B, A, n);
  tile_kernel<true, true><<<items, 1024>>>(g, A, B, ntx, nty, chunk);
  CK(hipDeviceSynchronize());
  ok2 = same6(B, R, n, "2-step tile (prefetch) vs naive") && ok2;
  F6 T = S;  // scratch
  copy6(T, A, n);
  copy6(B, A, n);
  tile_kernel<false><<<items, 1024>>>(g, A, B, ntx, nty, chunk);
  copy6(T, B, n);
  tile_kernel<false><<<items, 1024>>>(g, B, T, ntx, nty, chunk);
  CK(hipDeviceSynchronize());
  const bool ok1 = same6(T, R, n, "1-step tile x2 vs naive");
  printf("parity: 2-step %s, 1-step %s\n", ok2 ? "bitwise" : "DIFFERS", ok1 ? "bitwise" : "DIFFERS");
  // timing (ping-pong A <-> B; boundaries identical in both)
  copy6(B, A, n);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double cells = double(N - 4) * (N - 4) * (N - 4);
  auto launch = [&](int v, F6 src, F6 dst) {
    if (v == 0) tile_kernel<false><<<items, 1024>>>(g, src, dst, ntx, nty, chunk);
    if (v == 1) tile_kernel<true><<<items, 1024>>>(g, src, dst, ntx, nty, chunk);
    if (v == 2) tile_kernel<false, true><<<items, 1024>>>(g, src, dst, ntx, nty, chunk);
    if (v == 3) tile_kernel<true, true><<<items, 1024>>>(g, src, dst, ntx, nty, chunk);
    if (v == 5) tile_kernel<true, true, 56, 4, -52><<<items56, 1024>>>(g, src, dst, ntx56, nty, chunk);
  };
  {  // parity of the 56-wide shape
    copy6(B, A, n);
    launch(5, A, B);
    CK(hipDeviceSynchronize());
    printf("parity: 2-step 56-wide %s\n", same6(B, R, n, "2-step 56-wide vs naive") ? "bitwise" : "DIFFERS");
    copy6(B, A, n);
  }
  for (int v = 0; v < 6; v++) {
    if (v == 4) continue;
    const int two = v & 1;
    for (int wu = 0; wu < 2; wu++) launch(v, A, B);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) {
      F6 src = (r & 1) ? B : A, dst = (r & 1) ? A : B;
      launch(v, src, dst);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps, steps = two ? 2.0 : 1.0;
    printf("%s%s%s: %.4f ms per launch, %.1f G cell-steps/s (%d^3, chunk %d, %d items), "
           "algorithmic 96 B/cell-step -> %.2f TB/s equivalent\n",
           two ? "2-step" : "1-step", v >= 2 ? " (prefetch)" : "", v == 5 ? " 56-wide" : "", per, cells * steps / per / 1e6, N, chunk, v == 5 ? items56 : items,
           cells * steps * 96.0 / per / 1e9);
  }
  return ok1 && ok2 ? 0 : 2;
}
