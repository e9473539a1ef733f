// Which XCD does each workgroup land on?  (speed-only affinity check)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(unsigned *o) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  if (threadIdx.x == 0) o[blockIdx.x] = x;
}
int main() {
  const int nb = 512;
  unsigned *d;
  (void)hipMalloc(&d, nb * 4);
  k<<<nb, 1024>>>(d);
  std::vector<unsigned> h(nb);
  (void)hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
  int hist[16] = {0}, match = 0;
  for (int b = 0; b < nb; b++) {
    hist[h[b] & 15]++;
    if ((h[b] & 7) == (unsigned)((b + (h[0] & 7)) % 8)) match++;
  }
  for (int i = 0; i < 16; i++) printf("xcc %d: %d\n", i, hist[i]);
  printf("blocks matching (b + xcc0) %% 8: %d / %d\nfirst 16:", match, nb);
  for (int b = 0; b < 16; b++) printf(" %u", h[b]);
  printf("\n");
  return 0;
}
