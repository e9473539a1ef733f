// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the product kernels use (4, 8, 16 B per lane), on a 1 GiB stream.
#include <hip/hip_runtime.h>
#include <cstdio>
template <typename T>
__global__ void rd(const T *p, long long n, T *sink) {
  T acc{};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) acc += p[i];
  if (acc == T(12345)) *sink = acc;
}
struct d2 { double a, b; __device__ d2 &operator+=(const d2 &o) { a += o.a; b += o.b; return *this; } __device__ bool operator==(const d2 &o) const { return a == o.a; } __device__ d2() : a(0), b(0) {} __device__ d2(int v) : a(v), b(v) {} };
template <typename T>
__global__ void wr(T *p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) p[i] = T(1);
}
int main() {
  const long long bytes = 1LL << 30;
  char *buf, *sink;
  hipMalloc(&buf, bytes); hipMalloc(&sink, 64); hipMemset(buf, 0, bytes);
  for (int r = 0; r < 2; r++) {
    rd<unsigned><<<4096, 256>>>((const unsigned *)buf, bytes / 4, (unsigned *)sink);
    rd<double><<<4096, 256>>>((const double *)buf, bytes / 8, (double *)sink);
    rd<d2><<<4096, 256>>>((const d2 *)buf, bytes / 16, (d2 *)sink);
    wr<unsigned><<<4096, 256>>>((unsigned *)buf, bytes / 4);
    wr<double><<<4096, 256>>>((double *)buf, bytes / 8);
  }
  hipDeviceSynchronize();
  printf("done: each kernel streams %lld bytes (1 GiB); rd<u32>, rd<f64>, rd<16B>, wr<u32>, wr<f64>\n", bytes);
  return 0;
}
