// Microbenchmark: cost of a kernel that reads data produced by device-scope atomics in the
// previous kernel (vs plain stores), for 1-block and 2048-block consumers.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void prod_atomic(unsigned* buf, int nbins) {
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) atomicAdd(&buf[b], 1u);
}
__global__ void prod_plain(unsigned* buf, int nbins) {
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) buf[b] = buf[b] + 1u;
}
__global__ void prod_none(unsigned* buf, int nbins) {}
// consumer: every block reads the bins (vector) + a scalar word, writes one word
__global__ void cons_vec(const unsigned* buf, int nbins, unsigned* out) {
  unsigned s = 0;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) s += buf[b];
  s += buf[0];  // uniform -> scalar load
  if (s == 0xFFFFFFFFu) out[blockIdx.x] = s;
}
int main() {
  unsigned *buf, *out;
  CK(hipMalloc(&buf, 1 << 20)); CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 0, 1 << 20));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int nb = 257;
  for (int pblocks : {1, 64, 2048}) for (int cgrid : {1, 2048}) for (int mode = 0; mode < 3; ++mode) {
    for (int w = 0; w < 3; ++w) {
      if (mode == 0) prod_atomic<<<pblocks, 256>>>(buf, nb);
      else if (mode == 1) prod_plain<<<pblocks, 256>>>(buf, nb);
      else prod_none<<<pblocks, 256>>>(buf, nb);
      cons_vec<<<cgrid, 256>>>(buf, nb, out);
    }
    CK(hipDeviceSynchronize());
    const int R = 200;
    CK(hipEventRecord(e0));
    for (int r = 0; r < R; ++r) {
      if (mode == 0) prod_atomic<<<pblocks, 256>>>(buf, nb);
      else if (mode == 1) prod_plain<<<pblocks, 256>>>(buf, nb);
      else prod_none<<<pblocks, 256>>>(buf, nb);
      cons_vec<<<cgrid, 256>>>(buf, nb, out);
    }
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("producer %-6s pblocks %5d consumer grid %5d : %.2f us per pair\n",
           mode == 0 ? "atomic" : (mode == 1 ? "plain" : "none"), pblocks, cgrid, ms * 1000 / R);
  }
  return 0;
}
