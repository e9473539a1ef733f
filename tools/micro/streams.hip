// Placement sensitivity probe: NA arrays of 1.1 GB (512^3 fields), one kernel
// that reads R of them and writes W at the same index (the fused step's access
// pattern without the stencil).  Prints GB/s per trial; run it in several
// processes to see whether bandwidth depends on the physical pages obtained.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void streams(const double *const *in, double *const *out, int R, int W, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    double s = 0;
    for (int r = 0; r < R; r++) s += in[r][i];
    for (int w = 0; w < W; w++) out[w][i] = s + w;
  }
}

int main(int argc, char **argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 6, W = argc > 2 ? atoi(argv[2]) : 4;
  const size_t n = (size_t)528 * 513 * 513;
  const int mode = argc > 3 ? atoi(argv[3]) : 0;  // 0 separate, 1 arena, 2 contiguous, 3 uncached
  std::vector<double *> a(R + W);
  if (mode == 1) {
    double *base;
    if (hipMalloc(&base, n * 8 * (R + W)) != hipSuccess) return 1;
    for (int k = 0; k < R + W; k++) a[k] = base + (size_t)k * n;
  } else {
    for (auto &p : a) {
      hipError_t e = mode == 2 ? hipExtMallocWithFlags((void **)&p, n * 8, hipDeviceMallocContiguous)
                   : mode == 3 ? hipExtMallocWithFlags((void **)&p, n * 8, hipDeviceMallocUncached)
                               : hipMalloc(&p, n * 8);
      if (e != hipSuccess) { printf("alloc failed %d\n", (int)e); return 1; }
    }
  }
  for (auto &p : a) (void)hipMemset(p, 0, n * 8);
  double **din, **dout;
  (void)hipMalloc(&din, R * sizeof(double *));
  (void)hipMalloc(&dout, W * sizeof(double *));
  (void)hipMemcpy(din, a.data(), R * sizeof(double *), hipMemcpyHostToDevice);
  (void)hipMemcpy(dout, a.data() + R, W * sizeof(double *), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int t = 0; t < 4; t++) {
    (void)hipEventRecord(e0, 0);
    for (int k = 0; k < 5; k++) streams<<<256 * 16, 256>>>(din, dout, R, W, n);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%.1f ", 5.0 * n * 8 * (R + W) / (ms * 1e-3) / 1e9);
  }
  printf("GB/s\n");
  return 0;
}
