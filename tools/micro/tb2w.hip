// Two-step prototype, round 6: footprint shapes of the two-step kernel
// measured outside the product.  The product's tb2_kernel runs 64 x 16 lanes for 60 x 12 own
// points: its reads are ~1.9x the algorithmic bytes (x: 5 lines of 128 B per row for 60 own
// columns; y: 16 rows for 12; z: three halo planes per chunk).  Variants here:
//   PX = 1: one column per lane (the product's shape, x neighbours by DPP instead of LDS)
//   PX = 2: two adjacent columns per lane (16-B loads), 128 x 16 lanes for up to 124 x 12 own
// Arithmetic is the product's lean two-step body, operand for operand (E = chi1inv * D through
// a palette word per cell; B = b - C * (((a_p - a) + c) - c_p); D likewise), so every variant
// is checked bitwise against a naive one-point-per-thread pair of steps.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/micro/bin/tb2w tools/micro/tb2w.hip
//   tools/micro/bin/tb2w [N=512] [tz=48] [reps=10] [variant mask=3]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef const double __attribute__((address_space(1))) *gdp;
typedef const unsigned __attribute__((address_space(1))) *gup;
typedef double d2v __attribute__((ext_vector_type(2)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
constexpr unsigned OOB = 0xFFFFFFF0u;

__device__ __forceinline__ gdp sgpr_ptr(const void *p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (gdp)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double ld1(gdp p, unsigned off) {
  return *(gdp)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ d2v ld2(gdp p, unsigned off) {
  return *(const d2v __attribute__((address_space(1))) *)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ unsigned ldu1(gup p, unsigned off) {
  return *(gup)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ u2v ldu2(gup p, unsigned off) {
  return *(const u2v __attribute__((address_space(1))) *)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc_at(unsigned long long v, unsigned nrec) {
  asm volatile("" : "+s"(v));
  return __builtin_amdgcn_make_buffer_rsrc((void *)v, 0, (int)nrec, 0x00020000);
}
__device__ __forceinline__ void st1(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), r, off, 0, 0);
}
__device__ __forceinline__ void st2(__amdgpu_buffer_rsrc_t r, unsigned off, double a, double b) {
  u4v q;
  const u2v x = __builtin_bit_cast(u2v, a), y = __builtin_bit_cast(u2v, b);
  q.x = x.x, q.y = x.y, q.z = y.x, q.w = y.y;
  __builtin_amdgcn_raw_buffer_store_b128(q, r, off, 0, 0);
}
// lane i <- lane i + 1 (DPP wave_shl:1) / lane i <- lane i - 1 (wave_shr:1); the end lane keeps x
__device__ __forceinline__ double lane_next(double x) {
  const u2v u = __builtin_bit_cast(u2v, x);
  u2v r;
  r.x = __builtin_amdgcn_update_dpp((int)u.x, (int)u.x, 0x130, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp((int)u.y, (int)u.y, 0x130, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double lane_prev(double x) {
  const u2v u = __builtin_bit_cast(u2v, x);
  u2v r;
  r.x = __builtin_amdgcn_update_dpp((int)u.x, (int)u.x, 0x138, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp((int)u.y, (int)u.y, 0x138, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}

struct Item {
  int x;   // x0 | x1 << 16 own columns
  int y;   // y0 | y1 << 16
  int z;   // zs | ze << 16
  int lx;  // column of lane 0's first column
  unsigned uw;  // palette word uniform over the footprint, or ~0u
};
struct Args {
  int N;
  double C;
  const double *Do[3], *Bo[3];
  double *Dn[3], *Bn[3];
  const unsigned *uidx;
  const double *utab;
  const Item *items;
  int nitems;
  int qoff[9];  // PERS == 2: queue g holds items [qoff[g], qoff[g + 1])
};

constexpr int LY = 16, HY = 2;

// y-neighbour planes, row-major over 8 slots (E^n z, x; E^{n+1} z, x; B^{n+1} z, x; B^{n+2} z, x):
// rows 0 and LY + 1 are padding, so every access of a lane is a constant offset (< 64 KB, the
// ds offset field) from one per-lane address
template <int PX>
struct alignas(16) LdsT {
  double s[LY + 2][8][64 * PX];
};
enum { E1Z, E1X, E2Z, E2X, H1Z, H1X, H2Z, H2X };

// value of column j + 1 (x + 1) / j - 1 of this lane's PX columns
template <int PX>
__device__ __forceinline__ void xnext(const double (&v)[PX], double (&o)[PX]) {
  if (PX == 1) {
    o[0] = lane_next(v[0]);
  } else {
    o[0] = v[1];
    o[PX - 1] = lane_next(v[0]);
  }
}
template <int PX>
__device__ __forceinline__ void xprev(const double (&v)[PX], double (&o)[PX]) {
  if (PX == 1) {
    o[0] = lane_prev(v[0]);
  } else {
    o[PX - 1] = v[0];
    o[0] = lane_prev(v[PX - 1]);
  }
}

// this lane's PX doubles at LDS offset o (PX = 2: one 16-byte access, whose offset field is
// 16 bits wide; paired 8-byte accesses would merge into ds_*2_b64, whose 8-bit offsets cannot
// hold the slot offsets and cost an address register each)
template <int PX>
__device__ __forceinline__ void lds_put(double *bp, int o, const double (&v)[PX]) {
  if (PX == 1) {
    bp[o] = v[0];
  } else {
    d2v t;
    t.x = v[0], t.y = v[PX - 1];
    *(d2v *)(bp + o) = t;
  }
}
template <int PX>
__device__ __forceinline__ void lds_get(const double *bp, int o, double (&v)[PX]) {
  if (PX == 1) {
    v[0] = bp[o];
  } else {
    const d2v t = *(const d2v *)(bp + o);
    v[0] = t.x, v[PX - 1] = t.y;
  }
}

// BL: B(k) loaded after the B update of plane k - 1 (half a plane ahead) instead of with D(k+1)
template <int PX, bool UNI, bool BL, int DIST = 1>
__device__ __forceinline__ void body(const Args &a, const Item it, LdsT<PX> &L, const double (*sU)[256]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int x0 = it.x & 0xFFFF, x1 = it.x >> 16, y0 = it.y & 0xFFFF, y1 = it.y >> 16;
  const int zs = it.z & 0xFFFF, ze = it.z >> 16;
  const int N = a.N, zmax = N - 1;
  const int gx = it.lx + PX * lane, gy = y0 - HY + w;
  const int cx = min(max(gx, 0), N - PX), cy = min(max(gy, 0), N - 1);
  const unsigned col = (unsigned)((cx + cy * N) * 8);
  const unsigned s2 = (unsigned)((long long)N * N * 8);
  const double C = a.C;
  // with even lx and an even own width a lane's columns are both own or both not
  const bool own = gx >= x0 && gx + PX - 1 <= x1 && gy >= y0 && gy <= y1;
  const unsigned nrec = (unsigned)min((long long)N * N * N * 8, 0xFFFFFFFFLL);
  const unsigned long long pBn[3] = {(unsigned long long)sgpr_ptr(a.Bn[0]), (unsigned long long)sgpr_ptr(a.Bn[1]),
                                     (unsigned long long)sgpr_ptr(a.Bn[2])};
  const unsigned long long pDn[3] = {(unsigned long long)sgpr_ptr(a.Dn[0]), (unsigned long long)sgpr_ptr(a.Dn[1]),
                                     (unsigned long long)sgpr_ptr(a.Dn[2])};
  const gdp D0 = sgpr_ptr(a.Do[0]), D1 = sgpr_ptr(a.Do[1]), D2 = sgpr_ptr(a.Do[2]);
  const gdp B0 = sgpr_ptr(a.Bo[0]), B1 = sgpr_ptr(a.Bo[1]), B2 = sgpr_ptr(a.Bo[2]);
  const gup uix = (gup)sgpr_ptr(a.uidx);
  double cu[3] = {1, 1, 1};
  if (UNI) cu[0] = sU[0][it.uw & 255], cu[1] = sU[1][(it.uw >> 8) & 255], cu[2] = sU[2][(it.uw >> 16) & 255];
  struct Q {
    double d[3][PX], b[3][PX];
    unsigned ui[PX];
  };
  auto zc = [zmax](int z) { return min(max(z, 0), zmax); };
  auto ldd = [&](gdp p, unsigned o, double (&v)[PX]) {
    if (PX == 1) {
      v[0] = ld1(p, o);
    } else {
      const d2v t = ld2(p, o);
      v[0] = t.x, v[PX - 1] = t.y;
    }
  };
  auto ldw = [&](unsigned o, unsigned (&v)[PX]) {
    if (UNI) {
      for (int j = 0; j < PX; j++) v[j] = 0;
    } else if (PX == 1) {
      v[0] = ldu1(uix, o >> 1);
    } else {
      const u2v t = ldu2(uix, o >> 1);
      v[0] = t.x, v[PX - 1] = t.y;
    }
  };
  auto loadb = [&](int k, Q &q) {
    const unsigned ob = col + (unsigned)zc(k) * s2;
    ldd(B0, ob, q.b[0]);
    ldd(B1, ob, q.b[1]);
    ldd(B2, ob, q.b[2]);
  };
  auto load = [&](int k) -> Q {
    Q q;
    const unsigned o1 = col + (unsigned)zc(k + 1) * s2, ob = col + (unsigned)zc(k) * s2;
    ldd(D0, o1, q.d[0]);
    ldd(D1, o1, q.d[1]);
    ldd(D2, o1, q.d[2]);
    ldw(o1, q.ui);
    if (!BL) {
      ldd(B0, ob, q.b[0]);
      ldd(B1, ob, q.b[1]);
      ldd(B2, ob, q.b[2]);
    }
    return q;
  };
  auto uv = [&](unsigned ui, int c) -> double { return UNI ? cu[c] : sU[c][(ui >> (8 * c)) & 255]; };
  const int k0 = zs - 2;
  // carried across planes: D^n(k), B^{n+1}(k-1), D^{n+1}(k-1), B^{n+2}(k-2) x, y and the
  // palette words of k and k-1; E^n(k) = D^n(k) u(k) and E^{n+1}(k-1) = D^{n+1}(k-1) u(k-1)
  // are recomputed per plane (the same products, so the same values)
  double dn[3][PX];
  unsigned uk[PX], ukm[PX];
  {
    const unsigned o = col + (unsigned)zc(k0) * s2;
    ldd(D0, o, dn[0]);
    ldd(D1, o, dn[1]);
    ldd(D2, o, dn[2]);
    ldw(o, uk);
  }
  Q q = load(k0);
  Q q2;  // DIST 2: the plane after q (loaded two planes ahead of its use)
  if (DIST == 2) q2 = load(k0 + 1);
  Q qb;  // BL: B(k) loaded after the B update of plane k - 1
  if (BL) loadb(k0, qb);
  double b1[3][PX], d1[3][PX], h2x[PX], h2y[PX];
#pragma unroll
  for (int j = 0; j < PX; j++) {
    for (int c = 0; c < 3; c++) b1[c][j] = d1[c][j] = 0;
    h2x[j] = h2y[j] = 0;
    ukm[j] = uk[j];
  }
  const int lc = PX * lane;
  // this lane's LDS slot in row w (= padded row w + 1 is bp + R1)
  double *bp = &L.s[0][0][0] + (w * 8 * 64 * PX + lc);
  constexpr int RS = 8 * 64 * PX;
#define LO(row, slot) ((row) * RS + (slot) * 64 * PX)
  for (int k = k0; k <= ze; k++) {
    Q c = q;
    if (BL)
#pragma unroll
      for (int j = 0; j < PX; j++)
        for (int cc = 0; cc < 3; cc++) c.b[cc][j] = qb.b[cc][j];
    if (DIST == 2) {
      q = q2;
      q2 = load(min(k + 2, ze));
    } else {
      q = load(min(k + 1, ze));
    }
    double e1[2][PX], en[3][PX], f1[3][PX];  // E^n(k+1) x, y; E^n(k); E^{n+1}(k-1)
#pragma unroll
    for (int j = 0; j < PX; j++) {
#pragma unroll
      for (int cc = 0; cc < 2; cc++) e1[cc][j] = c.d[cc][j] * uv(c.ui[j], cc);
#pragma unroll
      for (int cc = 0; cc < 3; cc++) en[cc][j] = dn[cc][j] * uv(uk[j], cc), f1[cc][j] = d1[cc][j] * uv(ukm[j], cc);
    }
    lds_put<PX>(bp, LO(1, E1Z), en[2]);
    lds_put<PX>(bp, LO(1, E1X), en[0]);
    lds_put<PX>(bp, LO(1, E2Z), f1[2]);
    lds_put<PX>(bp, LO(1, E2X), f1[0]);
    __syncthreads();
    // step n at plane k: B^{n+1}(k)
    double Bx[PX], By[PX], Bz[PX], ezx[PX], eyx[PX], ezy[PX], exy[PX];
    xnext<PX>(en[2], ezx);
    xnext<PX>(en[1], eyx);
    lds_get<PX>(bp, LO(2, E1Z), ezy);
    lds_get<PX>(bp, LO(2, E1X), exy);
#pragma unroll
    for (int j = 0; j < PX; j++) {
      Bx[j] = c.b[0][j] - C * (ezy[j] - en[2][j] + en[1][j] - e1[1][j]);
      By[j] = c.b[1][j] - C * (e1[0][j] - en[0][j] + en[2][j] - ezx[j]);
      Bz[j] = c.b[2][j] - C * (eyx[j] - en[1][j] + en[0][j] - exy[j]);
    }
    lds_put<PX>(bp, LO(1, H1Z), Bz);
    lds_put<PX>(bp, LO(1, H1X), Bx);
    if (BL) loadb(min(k + 1, ze), qb);
    __syncthreads();
    double Dx[PX], Dy[PX], Dz[PX], Ex[PX], Ey[PX], hzx[PX], hyx[PX], hzy[PX], hxy[PX];
    xprev<PX>(Bz, hzx);
    xprev<PX>(By, hyx);
    lds_get<PX>(bp, LO(0, H1Z), hzy);
    lds_get<PX>(bp, LO(0, H1X), hxy);
#pragma unroll
    for (int j = 0; j < PX; j++) {
      Dx[j] = dn[0][j] - C * (hzy[j] - Bz[j] + By[j] - b1[1][j]);
      Dy[j] = dn[1][j] - C * (b1[0][j] - Bx[j] + Bz[j] - hzx[j]);
      Dz[j] = dn[2][j] - C * (hyx[j] - By[j] + Bx[j] - hxy[j]);
      Ex[j] = Dx[j] * uv(uk[j], 0), Ey[j] = Dy[j] * uv(uk[j], 1);
    }
    // step n+1 at plane k-1
    double Fx[PX], Fy[PX], Fz[PX], fzx[PX], fyx[PX], fzy[PX], fxy[PX];
    xnext<PX>(f1[2], fzx);
    xnext<PX>(f1[1], fyx);
    lds_get<PX>(bp, LO(2, E2Z), fzy);
    lds_get<PX>(bp, LO(2, E2X), fxy);
#pragma unroll
    for (int j = 0; j < PX; j++) {
      Fx[j] = b1[0][j] - C * (fzy[j] - f1[2][j] + f1[1][j] - Ey[j]);
      Fy[j] = b1[1][j] - C * (Ex[j] - f1[0][j] + f1[2][j] - fzx[j]);
      Fz[j] = b1[2][j] - C * (fyx[j] - f1[1][j] + f1[0][j] - fxy[j]);
    }
    lds_put<PX>(bp, LO(1, H2Z), Fz);
    lds_put<PX>(bp, LO(1, H2X), Fx);
    __syncthreads();
    double Gx[PX], Gy[PX], Gz[PX], gzx[PX], gyx[PX], gzy[PX], gxy[PX];
    xprev<PX>(Fz, gzx);
    xprev<PX>(Fy, gyx);
    lds_get<PX>(bp, LO(0, H2Z), gzy);
    lds_get<PX>(bp, LO(0, H2X), gxy);
#pragma unroll
    for (int j = 0; j < PX; j++) {
      Gx[j] = d1[0][j] - C * (gzy[j] - Fz[j] + Fy[j] - h2y[j]);
      Gy[j] = d1[1][j] - C * (h2x[j] - Fx[j] + Fz[j] - gzx[j]);
      Gz[j] = d1[2][j] - C * (gyx[j] - Fy[j] + Fx[j] - gxy[j]);
    }
    {
      const bool st = own && k - 1 >= zs && k - 1 < ze;
      const unsigned os = st ? col + (unsigned)(k - 1) * s2 : OOB;
      if (PX == 1) {
        st1(brsrc_at(pBn[0], nrec), os, Fx[0]);
        st1(brsrc_at(pBn[1], nrec), os, Fy[0]);
        st1(brsrc_at(pBn[2], nrec), os, Fz[0]);
        st1(brsrc_at(pDn[0], nrec), os, Gx[0]);
        st1(brsrc_at(pDn[1], nrec), os, Gy[0]);
        st1(brsrc_at(pDn[2], nrec), os, Gz[0]);
      } else {
        st2(brsrc_at(pBn[0], nrec), os, Fx[0], Fx[PX - 1]);
        st2(brsrc_at(pBn[1], nrec), os, Fy[0], Fy[PX - 1]);
        st2(brsrc_at(pBn[2], nrec), os, Fz[0], Fz[PX - 1]);
        st2(brsrc_at(pDn[0], nrec), os, Gx[0], Gx[PX - 1]);
        st2(brsrc_at(pDn[1], nrec), os, Gy[0], Gy[PX - 1]);
        st2(brsrc_at(pDn[2], nrec), os, Gz[0], Gz[PX - 1]);
      }
    }
#pragma unroll
    for (int j = 0; j < PX; j++) {
      h2x[j] = Fx[j], h2y[j] = Fy[j];
      b1[0][j] = Bx[j], b1[1][j] = By[j], b1[2][j] = Bz[j];
      d1[0][j] = Dx[j], d1[1][j] = Dy[j], d1[2][j] = Dz[j];
      for (int cc = 0; cc < 3; cc++) dn[cc][j] = c.d[cc][j];
      ukm[j] = uk[j], uk[j] = c.ui[j];
    }
  }
}

// PERS = 1: persistent workgroups taking items from one atomic counter (the product's tb2_kernel
// scheme); PERS = 2: persistent, one queue per XCD (the workgroup's XCC_ID picks its queue; an
// empty queue sends it to the next ones); PERS = 0: one workgroup per item in list order (the
// hardware deals consecutive workgroups to consecutive XCDs, so the list order decides which
// items share an L2)
template <int PX, bool BL, int PERS, int TAG>
__global__ __launch_bounds__(1024) void tbw_kernel(Args a, unsigned *ctr) {
  __shared__ double sU[3][256];
  __shared__ LdsT<PX> L;
  __shared__ int s_idx;
  for (int i = threadIdx.x; i < 3 * 256; i += 1024) sU[i >> 8][i & 255] = a.utab[i];
  unsigned xcc = 0;
  if (PERS == 2) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  int q0 = 0;  // PERS == 2: the queue being drained (own first)
  for (int it0 = blockIdx.x;;) {
    if (PERS == 1) {
      if (threadIdx.x == 0) {
        const unsigned v = atomicAdd(ctr, 1u);
        s_idx = v < (unsigned)a.nitems ? (int)v : -1;
      }
    } else if (PERS == 2) {
      if (threadIdx.x == 0) {
        int got = -1;
        for (; q0 < 8 && got < 0; q0++) {
          const int q = (int)((xcc + q0) & 7);
          const unsigned n = (unsigned)(a.qoff[q + 1] - a.qoff[q]);
          const unsigned v = atomicAdd(ctr + 32 * q, 1u);
          if (v < n) {
            got = a.qoff[q] + (int)v;
            break;
          }
        }
        s_idx = got;
      }
    }
    __syncthreads();
    const int idx = PERS ? s_idx : it0;
    if (idx < 0) break;
    const Item it = a.items[idx];
    if (__builtin_amdgcn_readfirstlane(it.uw) != ~0u)
      body<PX, true, BL, (TAG >= 100 ? 2 : 1)>(a, it, L, sU);
    else
      body<PX, false, BL, (TAG >= 100 ? 2 : 1)>(a, it, L, sU);
    if (!PERS) break;
    __syncthreads();
  }
}

// ---- three steps per z-march (one column per lane, 64 x 16 lanes for 58 x 10 own points):
// step n at plane k, step n+1 at plane k-1, step n+2 at plane k-2; per three steps a point's D,
// B are read once and written once.  The same operand order as the two-step body.
constexpr int HY3 = 3;
struct alignas(16) LdsT3 {
  double s[LY + 2][12][64];  // slots 0-5: E^n, E^{n+1}, E^{n+2} (z, x); 6-11: B^{n+1..n+3} (z, x)
};
template <bool UNI>
__device__ __forceinline__ void body3(const Args &a, const Item it, LdsT3 &L, const double (*sU)[256]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int x0 = it.x & 0xFFFF, x1 = it.x >> 16, y0 = it.y & 0xFFFF, y1 = it.y >> 16;
  const int zs = it.z & 0xFFFF, ze = it.z >> 16;
  const int N = a.N, zmax = N - 1;
  const int gx = it.lx + lane, gy = y0 - HY3 + w;
  const int cx = min(max(gx, 0), N - 1), cy = min(max(gy, 0), N - 1);
  const unsigned col = (unsigned)((cx + cy * N) * 8);
  const unsigned s2 = (unsigned)((long long)N * N * 8);
  const double C = a.C;
  const bool own = gx >= x0 && gx <= x1 && gy >= y0 && gy <= y1;
  const unsigned nrec = (unsigned)min((long long)N * N * N * 8, 0xFFFFFFFFLL);
  const unsigned long long pBn[3] = {(unsigned long long)sgpr_ptr(a.Bn[0]), (unsigned long long)sgpr_ptr(a.Bn[1]),
                                     (unsigned long long)sgpr_ptr(a.Bn[2])};
  const unsigned long long pDn[3] = {(unsigned long long)sgpr_ptr(a.Dn[0]), (unsigned long long)sgpr_ptr(a.Dn[1]),
                                     (unsigned long long)sgpr_ptr(a.Dn[2])};
  const gdp D0 = sgpr_ptr(a.Do[0]), D1 = sgpr_ptr(a.Do[1]), D2 = sgpr_ptr(a.Do[2]);
  const gdp B0 = sgpr_ptr(a.Bo[0]), B1 = sgpr_ptr(a.Bo[1]), B2 = sgpr_ptr(a.Bo[2]);
  const gup uix = (gup)sgpr_ptr(a.uidx);
  double cu0 = 1, cu1 = 1, cu2 = 1;
  if (UNI) cu0 = sU[0][it.uw & 255], cu1 = sU[1][(it.uw >> 8) & 255], cu2 = sU[2][(it.uw >> 16) & 255];
  auto uv = [&](unsigned ui, int c) -> double {
    if (UNI) return c == 0 ? cu0 : (c == 1 ? cu1 : cu2);
    return sU[c][(ui >> (8 * c)) & 255];
  };
  struct Q {
    double d0, d1, d2, b0, b1, b2;
    unsigned ui;
  };
  auto zc = [zmax](int z) { return min(max(z, 0), zmax); };
  auto load = [&](int k) -> Q {
    Q q;
    const unsigned o1 = col + (unsigned)zc(k + 1) * s2, ob = col + (unsigned)zc(k) * s2;
    q.d0 = ld1(D0, o1), q.d1 = ld1(D1, o1), q.d2 = ld1(D2, o1);
    q.ui = UNI ? 0u : ldu1(uix, o1 >> 1);
    q.b0 = ld1(B0, ob), q.b1 = ld1(B1, ob), q.b2 = ld1(B2, ob);
    return q;
  };
  const int k0 = zs - 3;
  double dn0, dn1, dn2;
  unsigned uk, u1, u2;
  {
    const unsigned o = col + (unsigned)zc(k0) * s2;
    dn0 = ld1(D0, o), dn1 = ld1(D1, o), dn2 = ld1(D2, o);
    uk = UNI ? 0u : ldu1(uix, o >> 1);
    u1 = u2 = uk;
  }
  Q q = load(k0);
  double b1x = 0, b1y = 0, b1z = 0, d1x = 0, d1y = 0, d1z = 0;  // B^{n+1}(k-1), D^{n+1}(k-1)
  double b2x = 0, b2y = 0, b2z = 0, d2x = 0, d2y = 0, d2z = 0;  // B^{n+2}(k-2), D^{n+2}(k-2)
  double h3x = 0, h3y = 0;                                      // B^{n+3}(k-3) x, y
  double *bp = &L.s[0][0][0] + (w * 12 * 64 + lane);
#define L3(row, slot) bp[(row) * 12 * 64 + (slot) * 64]
  for (int k = k0; k <= ze + 1; k++) {
    const Q c = q;
    q = load(min(k + 1, ze + 1));
    const double enx = dn0 * uv(uk, 0), eny = dn1 * uv(uk, 1), enz = dn2 * uv(uk, 2);
    const double e1x = c.d0 * uv(c.ui, 0), e1y = c.d1 * uv(c.ui, 1);
    const double f1x = d1x * uv(u1, 0), f1y = d1y * uv(u1, 1), f1z = d1z * uv(u1, 2);
    const double g2x = d2x * uv(u2, 0), g2y = d2y * uv(u2, 1), g2z = d2z * uv(u2, 2);
    L3(1, 0) = enz, L3(1, 1) = enx, L3(1, 2) = f1z, L3(1, 3) = f1x;
    L3(1, 4) = g2z, L3(1, 5) = g2x;
    __syncthreads();
    // step n at k
    const double Bx = c.b0 - C * (L3(2, 0) - enz + eny - e1y);
    const double By = c.b1 - C * (e1x - enx + enz - lane_next(enz));
    const double Bz = c.b2 - C * (lane_next(eny) - eny + enx - L3(2, 1));
    // the y-neighbours of E^{n+1}(k-1) and E^{n+2}(k-2) (written at the top of this plane)
    const double g2zy = L3(2, 4), g2xy = L3(2, 5);
    const double f1zy = L3(2, 2), f1xy = L3(2, 3);
    L3(1, 6) = Bz, L3(1, 7) = Bx;
    __syncthreads();
    const double Dx = dn0 - C * (L3(0, 6) - Bz + By - b1y);
    const double Dy = dn1 - C * (b1x - Bx + Bz - lane_prev(Bz));
    const double Dz = dn2 - C * (lane_prev(By) - By + Bx - L3(0, 7));
    const double Ex = Dx * uv(uk, 0), Ey = Dy * uv(uk, 1);
    // step n+1 at k-1
    const double Fx = b1x - C * (f1zy - f1z + f1y - Ey);
    const double Fy = b1y - C * (Ex - f1x + f1z - lane_next(f1z));
    const double Fz = b1z - C * (lane_next(f1y) - f1y + f1x - f1xy);
    L3(1, 8) = Fz, L3(1, 9) = Fx;
    __syncthreads();
    const double Gx = d1x - C * (L3(0, 8) - Fz + Fy - b2y);
    const double Gy = d1y - C * (b2x - Fx + Fz - lane_prev(Fz));
    const double Gz = d1z - C * (lane_prev(Fy) - Fy + Fx - L3(0, 9));
    const double Gex = Gx * uv(u1, 0), Gey = Gy * uv(u1, 1);
    // step n+2 at k-2
    const double Kx = b2x - C * (g2zy - g2z + g2y - Gey);
    const double Ky = b2y - C * (Gex - g2x + g2z - lane_next(g2z));
    const double Kz = b2z - C * (lane_next(g2y) - g2y + g2x - g2xy);
    L3(1, 10) = Kz, L3(1, 11) = Kx;
    __syncthreads();
    const double Mx = d2x - C * (L3(0, 10) - Kz + Ky - h3y);
    const double My = d2y - C * (h3x - Kx + Kz - lane_prev(Kz));
    const double Mz = d2z - C * (lane_prev(Ky) - Ky + Kx - L3(0, 11));
    {
      const bool st = own && k - 2 >= zs && k - 2 < ze;
      const unsigned os = st ? col + (unsigned)(k - 2) * s2 : OOB;
      st1(brsrc_at(pBn[0], nrec), os, Kx);
      st1(brsrc_at(pBn[1], nrec), os, Ky);
      st1(brsrc_at(pBn[2], nrec), os, Kz);
      st1(brsrc_at(pDn[0], nrec), os, Mx);
      st1(brsrc_at(pDn[1], nrec), os, My);
      st1(brsrc_at(pDn[2], nrec), os, Mz);
    }
    h3x = Kx, h3y = Ky;
    b2x = Fx, b2y = Fy, b2z = Fz, d2x = Gx, d2y = Gy, d2z = Gz, u2 = u1;
    b1x = Bx, b1y = By, b1z = Bz, d1x = Dx, d1y = Dy, d1z = Dz, u1 = uk;
    dn0 = c.d0, dn1 = c.d1, dn2 = c.d2, uk = c.ui;
  }
#undef L3
}

template <int TAG>
__global__ __launch_bounds__(1024) void tbw3_kernel(Args a, unsigned *ctr) {
  __shared__ double sU[3][256];
  __shared__ LdsT3 L;
  __shared__ int s_idx;
  for (int i = threadIdx.x; i < 3 * 256; i += 1024) sU[i >> 8][i & 255] = a.utab[i];
  for (;;) {
    if (threadIdx.x == 0) {
      const unsigned v = atomicAdd(ctr, 1u);
      s_idx = v < (unsigned)a.nitems ? (int)v : -1;
    }
    __syncthreads();
    const int idx = s_idx;
    if (idx < 0) break;
    const Item it = a.items[idx];
    if (__builtin_amdgcn_readfirstlane(it.uw) != ~0u)
      body3<true>(a, it, L, sU);
    else
      body3<false>(a, it, L, sU);
    __syncthreads();
  }
}

// ---- naive pair of steps over [2, N-3]^3 (the same expressions, one point per thread)
struct NArgs {
  int N;
  double C;
  const double *D[3], *B[3];
  double *Dt[3], *Bt[3];
  const unsigned *uidx;
  const double *utab;
};
__device__ __forceinline__ double nu(const NArgs &a, long long p, int c) {
  return a.utab[c * 256 + ((a.uidx[p] >> (8 * c)) & 255)];
}
__global__ void naive_b(NArgs a) {
  const long long N = a.N, n = N * N * N;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < n; p += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(p % N), j = (int)((p / N) % N), k = (int)(p / (N * N));
    if (i < 2 || j < 2 || k < 2 || i > N - 3 || j > N - 3 || k > N - 3) {
      for (int c = 0; c < 3; c++) a.Bt[c][p] = a.B[c][p];
      continue;
    }
    auto E = [&](int c, long long q) { return a.D[c][q] * nu(a, q, c); };
    const long long px = p + 1, py = p + N, pz = p + N * N;
    a.Bt[0][p] = a.B[0][p] - a.C * (E(2, py) - E(2, p) + E(1, p) - E(1, pz));
    a.Bt[1][p] = a.B[1][p] - a.C * (E(0, pz) - E(0, p) + E(2, p) - E(2, px));
    a.Bt[2][p] = a.B[2][p] - a.C * (E(1, px) - E(1, p) + E(0, p) - E(0, py));
  }
}
__global__ void naive_d(NArgs a) {  // reads Bt (new), D; writes Dt
  const long long N = a.N, n = N * N * N;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < n; p += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(p % N), j = (int)((p / N) % N), k = (int)(p / (N * N));
    if (i < 2 || j < 2 || k < 2 || i > N - 3 || j > N - 3 || k > N - 3) {
      for (int c = 0; c < 3; c++) a.Dt[c][p] = a.D[c][p];
      continue;
    }
    const long long mx = p - 1, my = p - N, mz = p - N * N;
    auto H = [&](int c, long long q) { return a.Bt[c][q]; };
    a.Dt[0][p] = a.D[0][p] - a.C * (H(2, my) - H(2, p) + H(1, p) - H(1, mz));
    a.Dt[1][p] = a.D[1][p] - a.C * (H(0, mz) - H(0, p) + H(2, p) - H(2, mx));
    a.Dt[2][p] = a.D[2][p] - a.C * (H(1, mx) - H(1, p) + H(0, p) - H(0, my));
  }
}

__global__ void init_kernel(double *p, long long n, unsigned seed) {
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    unsigned long long x = (unsigned long long)q * 0x9E3779B97F4A7C15ULL + seed;
    x ^= x >> 31, x *= 0xBF58476D1CE4E5B9ULL, x ^= x >> 29;
    p[q] = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}
// palette word per cell: index 1 inside a waveguide core along x (|y - N/2|, |z - N/2| < 12),
// index 0 elsewhere (the headline's shape: most items uniform)
__global__ void init_u(unsigned *u, int N) {
  const long long n = (long long)N * N * N;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const int j = (int)((q / N) % N), k = (int)(q / ((long long)N * N));
    const bool core = abs(j - N / 2) < 12 && abs(k - N / 2) < 12;
    u[q] = core ? 0x010101u : 0u;
  }
}

struct F6 {
  double *d[3], *b[3];
};
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
// own region [lo, hi]^3 bitwise
static bool same_own(F6 a, F6 b, int N, int lo, int hi, const char *what) {
  const long long n = (long long)N * N * N;
  std::vector<double> x(n), y(n);
  bool ok = true;
  for (int c = 0; c < 6; c++) {
    CK(hipMemcpy(x.data(), c < 3 ? a.d[c] : a.b[c - 3], n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), c < 3 ? b.d[c] : b.b[c - 3], n * 8, hipMemcpyDeviceToHost));
    long long bad = 0;
    for (int k = lo; k <= hi; k++)
      for (int j = lo; j <= hi; j++)
        for (int i = lo; i <= hi; i++) {
          const long long q = i + (long long)N * (j + (long long)N * k);
          bad += memcmp(&x[q], &y[q], 8) != 0;
        }
    if (bad) printf("%s: component %d differs at %lld points\n", what, c, bad), ok = false;
  }
  return ok;
}

// items over the own box [lo, hi]^3: x in widths of ow (the last narrower), y balanced rows of
// <= 12, z balanced chunks of <= tz; uniform palette word per item from the host copy.
// Order: xcd = false: z chunk, then tile row, then tile column (x fastest); xcd = true: the
// tiles (column-major: x, then y) cut into 8 equal runs, run g to XCD g (workgroup b of the
// list takes run b % 8's item b / 8, z chunk outer), so each XCD marches a y-band of tiles
// whose halo rows its L2 shares
static std::vector<Item> make_items(int N, int lo, int hi, int ow, int tz, const std::vector<unsigned> &u,
                                    int xcd, int *qoff = nullptr, int H = 2, int OR = 12) {
  const int W = hi - lo + 1, nty = (W + OR - 1) / OR, nch = (W + tz - 1) / tz, ntx = (W + ow - 1) / ow;
  auto mk = [&](int ch, int ty, int tx) {
    Item it;
    const int x0 = lo + ow * tx, x1 = std::min(x0 + ow - 1, hi);
    const int y0 = lo + W * ty / nty, y1 = lo + W * (ty + 1) / nty - 1;
    const int zs = lo + W * ch / nch, ze = lo + W * (ch + 1) / nch;
    it.x = x0 | (x1 << 16), it.y = y0 | (y1 << 16), it.z = zs | (ze << 16), it.lx = x0 - H;
    unsigned ref = u[(x0 - H) + (long long)N * ((y0 - H) + (long long)N * (zs - H))];
    bool uni = true;
    for (int k = zs - H; k <= ze + H - 1 && uni; k++)
      for (int j = y0 - H; j <= y1 + H && uni; j++)
        for (int i = x0 - H; i <= x1 + H; i++)
          if (u[i + (long long)N * (j + (long long)N * k)] != ref) {
            uni = false;
            break;
          }
    it.uw = uni ? ref : ~0u;
    return it;
  };
  std::vector<Item> v;
  if (!xcd) {
    for (int ch = 0; ch < nch; ch++)
      for (int ty = 0; ty < nty; ty++)
        for (int tx = 0; tx < ntx; tx++) v.push_back(mk(ch, ty, tx));
    return v;
  }
  const int nt = ntx * nty;
  std::vector<std::vector<Item>> g(8);
  if (xcd == 1) {
    for (int ch = 0; ch < nch; ch++)
      for (int t = 0; t < nt; t++) {
        const int tx = t / nty, ty = t % nty;  // column-major: a run is a y-band
        g[(long long)t * 8 / nt].push_back(mk(ch, ty, tx));
      }
  } else {  // xcd = 2: a 2 x 4 grid of tile blocks, block g to XCD g, row-major inside
    const int BX = 2, BY = 4;
    for (int gy = 0; gy < BY; gy++)
      for (int gx = 0; gx < BX; gx++)
        for (int ch = 0; ch < nch; ch++)
          for (int ty = nty * gy / BY; ty < nty * (gy + 1) / BY; ty++)
            for (int tx = ntx * gx / BX; tx < ntx * (gx + 1) / BX; tx++) g[gx + BX * gy].push_back(mk(ch, ty, tx));
  }
  if (qoff) {  // per-XCD queues: the lists one after another
    qoff[0] = 0;
    for (int x = 0; x < 8; x++) {
      v.insert(v.end(), g[x].begin(), g[x].end());
      qoff[x + 1] = (int)v.size();
    }
    return v;
  }
  size_t mx = 0;
  for (auto &q : g) mx = std::max(mx, q.size());
  for (size_t i = 0; i < mx; i++)
    for (int x = 0; x < 8; x++)
      if (i < g[x].size()) v.push_back(g[x][i]);  // unequal runs: the tail loses the mapping
  return v;
}

struct Variant {
  const char *name;
  int px, bl, pers, xcd, steps;
};

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 512;
  const int tz = argc > 2 ? atoi(argv[2]) : 48;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int rounds = argc > 4 ? atoi(argv[4]) : 3;
  const int lo = 16, hi = N - 17;  // the headline's L2 (512^3: 480 columns per axis)
  const long long n = (long long)N * N * N;
  if (N < 64 || (N & 1) || tz < 4) {
    fprintf(stderr, "bad shape\n");
    return 1;
  }
  F6 A = alloc6(n), B = alloc6(n), R = alloc6(n), S = alloc6(n), A0 = alloc6(n), R3 = alloc6(n);
  unsigned *du, *ctr;
  double *dt;
  CK(hipMalloc(&du, n * 4));
  CK(hipMalloc(&ctr, 8 * 32 * 4));
  CK(hipMalloc(&dt, 3 * 256 * 8));
  {
    std::vector<double> t(3 * 256, 1.0);
    for (int c = 0; c < 3; c++) t[c * 256 + 1] = 1.0 / 12.0;
    CK(hipMemcpy(dt, t.data(), t.size() * 8, hipMemcpyHostToDevice));
  }
  for (int c = 0; c < 3; c++) {
    init_kernel<<<4096, 256>>>(A.d[c], n, 11 + c);
    init_kernel<<<4096, 256>>>(A.b[c], n, 101 + c);
  }
  init_u<<<4096, 256>>>(du, N);
  CK(hipDeviceSynchronize());
  std::vector<unsigned> hu(n);
  CK(hipMemcpy(hu.data(), du, n * 4, hipMemcpyDeviceToHost));
  // naive reference: two steps A -> R
  {
    NArgs na{N, 0.5};
    for (int c = 0; c < 3; c++) na.D[c] = A.d[c], na.B[c] = A.b[c], na.Dt[c] = S.d[c], na.Bt[c] = S.b[c];
    na.uidx = du, na.utab = dt;
    naive_b<<<8192, 256>>>(na);
    naive_d<<<8192, 256>>>(na);
    NArgs nb = na;
    for (int c = 0; c < 3; c++) nb.D[c] = S.d[c], nb.B[c] = S.b[c], nb.Dt[c] = R.d[c], nb.Bt[c] = R.b[c];
    naive_b<<<8192, 256>>>(nb);
    naive_d<<<8192, 256>>>(nb);
    NArgs nc = na;  // a third step R -> R3
    for (int c = 0; c < 3; c++) nc.D[c] = R.d[c], nc.B[c] = R.b[c], nc.Dt[c] = R3.d[c], nc.Bt[c] = R3.b[c];
    naive_b<<<8192, 256>>>(nc);
    naive_d<<<8192, 256>>>(nc);
    CK(hipDeviceSynchronize());
  }
  copy6(A0, A, n);  // the timing loops ping-pong A <-> B: each variant starts from A0
  const Variant vs[] = {
      {"px1 pers", 1, 0, 1, 0, 2},   {"px2 bl pers", 2, 1, 1, 0, 2},   {"3-step px1 pers", 1, 0, 1, 0, 3},
  };


  const int nv = sizeof(vs) / sizeof(vs[0]);
  std::vector<Item *> di(nv);
  std::vector<int> ni(nv), nuni(nv);
  std::vector<std::vector<int>> qo(nv, std::vector<int>(9, 0));
  for (int v = 0; v < nv; v++) {
    const bool three = vs[v].steps == 3;
    std::vector<Item> items = make_items(N, lo, hi, three ? 58 : vs[v].px == 1 ? 60 : 124, tz, hu,
                                         vs[v].xcd, vs[v].pers == 2 ? qo[v].data() : nullptr,
                                         three ? 3 : 2, three ? 10 : 12);
    CK(hipMalloc(&di[v], items.size() * sizeof(Item)));
    CK(hipMemcpy(di[v], items.data(), items.size() * sizeof(Item), hipMemcpyHostToDevice));
    ni[v] = (int)items.size();
    nuni[v] = 0;
    for (auto &it : items) nuni[v] += it.uw != ~0u;
  }
  auto launch = [&](int v, F6 s, F6 t) {
    Args a{N, 0.5};
    for (int c = 0; c < 3; c++) a.Do[c] = s.d[c], a.Bo[c] = s.b[c], a.Dn[c] = t.d[c], a.Bn[c] = t.b[c];
    a.uidx = du, a.utab = dt, a.items = di[v], a.nitems = ni[v];
    for (int x = 0; x < 9; x++) a.qoff[x] = qo[v][x];
    const Variant &q = vs[v];
    const unsigned g = q.pers ? 256u : (unsigned)ni[v];
    if (q.pers) CK(hipMemsetAsync(ctr, 0, 8 * 32 * 4));
#define L_(PX, BL, P, T) tbw_kernel<PX, BL, (int)(P), T><<<g, 1024>>>(a, ctr)
    switch (v) {
      case 0: L_(1, false, 1, 0); break;
      case 1: L_(2, true, 1, 5); break;
      case 2: tbw3_kernel<0><<<g, 1024>>>(a, ctr); break;
    }
#undef L_
  };
  bool all = true;
  for (int v = 0; v < nv; v++) {  // parity of every variant
    copy6(A, A0, n);
    copy6(B, A, n);
    launch(v, A, B);
    CK(hipDeviceSynchronize());
    const bool ok = same_own(B, vs[v].steps == 3 ? R3 : R, N, lo, hi, vs[v].name);
    printf("%-12s %s (%d items, %d uniform)\n", vs[v].name, ok ? "bitwise" : "DIFFERS", ni[v], nuni[v]);
    all = all && ok;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double cells = double(hi - lo + 1) * (hi - lo + 1) * (hi - lo + 1);
  std::vector<std::vector<double>> ms(nv);
  for (int r = 0; r < rounds; r++)
    for (int q = 0; q < nv; q++) {
      const int v = (r & 1) ? nv - 1 - q : q;  // alternate the order
      for (int wu = 0; wu < 2; wu++) launch(v, A, B);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; i++) launch(v, (i & 1) ? B : A, (i & 1) ? A : B);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / reps);
    }
  for (int v = 0; v < nv; v++) {
    std::vector<double> x = ms[v];
    std::sort(x.begin(), x.end());
    const double med = x[x.size() / 2];
    printf("%-12s tz %d: median %.4f ms per launch (2 steps) [", vs[v].name, tz, med);
    for (double y : ms[v]) printf(" %.4f", y);
    printf(" ], %.1f G cell-steps/s, %.2f TB/s algorithmic (96 B per point per launch)\n",
           vs[v].steps * cells / med / 1e6, cells * 96.0 / med / 1e9);
  }
  return all ? 0 : 2;
}
