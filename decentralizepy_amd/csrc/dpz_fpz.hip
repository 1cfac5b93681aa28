// Block-floating fp32 value coding: the float leg of EliasFpzip / EliasFpzipLossy.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   compression/EliasFpzip.py:19-51       fpzip.compress(arr, precision=0)    (lossless)
//   compression/EliasFpzipLossy.py:14-58  fpzip.compress(arr, precision=p)    (lossy, p = 16)
// fpzip is absent from this image, so the byte format is this build's own (parity with fpzip's
// bytes is unpinned); the contract kept is fpzip's: precision 0 round-trips every fp32 bit
// pattern, precision p keeps the p most significant bits of each value's bit pattern (sign,
// exponent, p - 9 mantissa bits; the rest truncated; from p = 10 on a NaN stays a NaN).
//
// Format (little-endian 32-bit words):
//   header  [0] 'DPFZ' magic  [1] n  [2] precision (32 = lossless)  [3] nblk = ceil(n / 256)
//   table   nblk + 1 words: word offset of each block from the start of the block area; the last
//           entry is the block area's length
//   block   (256 values, the last one n - 256 (nblk - 1)):
//           [0] emin | w << 8 | mb << 16   (exponent base, exponent width 0..8, mantissa bits)
//           sign plane: 1 bit a value, exponent plane: w bits (e - emin), mantissa plane: mb bits,
//           each plane a LSB-first bit stream padded to whole words (value j at bits [j*b, j*b+b)).
// Top-k values of one block share a handful of exponents (w = 3..5), so the lossless stream is
// ~12 % below raw fp32 and the 16-bit lossy stream ~62 % below; the mantissas of trained weights
// are close to random, which is where fpzip's predictive coder ends up as well.
//
// Encode: 3 launches — size (one wave per block: exponent range -> block words), a 1-workgroup
// scan (table + header), pack (one wave per block assembles its planes in LDS, then stores them
// as whole words).  Decode: 1 launch, one wave per block, sync-free (n comes from the host copy
// of the header).
#include "dpz_common.h"

namespace dpz {

constexpr int FZ_B = 256;                      // values per block (4 per lane of one wave)
constexpr int FZ_MAXW = 1 + 8 + 8 * 8 + 8 * 23;  // words of a full block at w = 8, mb = 23
constexpr uint32_t FZ_MAGIC = 0x5A465044u;     // "DPFZ"
constexpr int64_t FZ_MAXN = int64_t(1) << 30;  // values a stream (block offsets stay 32-bit)

struct FzHdr {
  uint64_t words;   // block-area words
  uint64_t nbytes;  // whole stream
};

__device__ __forceinline__ int fz_bits(uint32_t v) { return v ? 32 - __clz(v) : 0; }

__device__ __forceinline__ uint32_t fz_words(int cnt, int w, int mb) {
  return 1u + (uint32_t)((cnt + 31) / 32) + (uint32_t)((cnt * w + 31) / 32) +
         (uint32_t)((cnt * mb + 31) / 32);
}

// the 4 values of this lane (block-relative j = 4 * lane + e); exponent range over the wave
__device__ __forceinline__ void fz_load(const float* __restrict__ x, int64_t n, int64_t b,
                                        int prec, int lane, uint32_t u[4], int* cnt_out,
                                        uint32_t* emin_out, int* w_out) {
  const int64_t base = b * FZ_B;
  const int cnt = (int)((n - base) < FZ_B ? (n - base) : FZ_B);
  const int64_t i0 = base + 4 * lane;
  if (4 * lane + 3 < cnt && aligned16(x)) {
    const float4 v = *reinterpret_cast<const float4*>(x + i0);
    u[0] = __float_as_uint(v.x); u[1] = __float_as_uint(v.y);
    u[2] = __float_as_uint(v.z); u[3] = __float_as_uint(v.w);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = (4 * lane + e < cnt) ? __float_as_uint(x[i0 + e]) : 0u;
  }
  if (prec < 32) {  // keep the top `prec` bits; from 10 bits on a NaN keeps a mantissa bit
    const uint32_t keep = ~((1u << (32 - prec)) - 1u);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t t = u[e] & keep;
      const bool nan = (u[e] & 0x7F800000u) == 0x7F800000u && (u[e] & 0x7FFFFFu) != 0u;
      u[e] = (prec >= 10 && nan && (t & 0x7FFFFFu) == 0u) ? (t | 0x400000u) : t;
    }
  }
  uint32_t lo = 255u, hi = 0u;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (4 * lane + e < cnt) {
      const uint32_t ex = (u[e] >> 23) & 0xFFu;
      lo = ex < lo ? ex : lo;
      hi = ex > hi ? ex : hi;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t l2 = __shfl_xor(lo, d, 64), h2 = __shfl_xor(hi, d, 64);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
  }
  *cnt_out = cnt;
  *emin_out = lo;
  *w_out = fz_bits(hi - lo);
}

__global__ void __launch_bounds__(256) fz_size_kernel(const float* __restrict__ x, int64_t n,
                                                      int64_t nblk, int prec, int mb,
                                                      uint32_t* __restrict__ blk_words) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nblk) return;
  const int lane = threadIdx.x & 63;
  uint32_t u[4], emin;
  int cnt, w;
  fz_load(x, n, b, prec, lane, u, &cnt, &emin, &w);
  if (lane == 0) blk_words[b] = fz_words(cnt, w, mb);
}

__global__ void __launch_bounds__(1024) fz_scan_kernel(int64_t n, int64_t nblk, int prec,
                                                       const uint32_t* __restrict__ blk_words,
                                                       uint32_t* __restrict__ out32,
                                                       FzHdr* hdr) {
  __shared__ uint64_t wsum[16];
  uint64_t carry = 0;
  uint32_t* table = out32 + 4;
  for (int64_t b0 = 0; b0 < nblk; b0 += 1024) {
    const int64_t b = b0 + threadIdx.x;
    const uint64_t v = b < nblk ? blk_words[b] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot) + carry;
    if (b < nblk) table[b] = (uint32_t)ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    table[nblk] = (uint32_t)carry;
    out32[0] = FZ_MAGIC;
    out32[1] = (uint32_t)n;
    out32[2] = (uint32_t)prec;
    out32[3] = (uint32_t)nblk;
    hdr->words = carry;
    hdr->nbytes = 4 * (4 + (uint64_t)nblk + 1 + carry);
  }
}

// OR `v` (at most 32 bits wide, `bits` of them) into the LDS bit stream at bit `pos`
__device__ __forceinline__ void fz_put(uint32_t* s, uint32_t pos, uint32_t v, int bits) {
  if (!bits) return;
  const uint32_t wi = pos >> 5, sh = pos & 31u;
  const uint64_t v64 = (uint64_t)v << sh;
  if ((uint32_t)v64) atomicOr(&s[wi], (uint32_t)v64);
  if (sh + bits > 32 && (uint32_t)(v64 >> 32)) atomicOr(&s[wi + 1], (uint32_t)(v64 >> 32));
}

__global__ void __launch_bounds__(256) fz_pack_kernel(const float* __restrict__ x, int64_t n,
                                                      int64_t nblk, int prec, int mb,
                                                      uint32_t* __restrict__ out32) {
  __shared__ uint32_t stage[4][FZ_MAXW + 1];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wid;
  if (b >= nblk) return;  // whole waves only: no block-wide barrier below
  uint32_t* s = stage[wid];
  for (int q = lane; q < FZ_MAXW + 1; q += 64) s[q] = 0u;
  uint32_t u[4], emin;
  int cnt, w;
  fz_load(x, n, b, prec, lane, u, &cnt, &emin, &w);
  const uint32_t ps = 1u, pe = ps + (uint32_t)((cnt + 31) / 32);
  const uint32_t pm = pe + (uint32_t)((cnt * w + 31) / 32);
  const uint32_t nw = pm + (uint32_t)((cnt * mb + 31) / 32);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t j = 4u * lane + e;
    if ((int)j < cnt) {
      fz_put(s + ps, j, u[e] >> 31, 1);
      fz_put(s + pe, j * w, ((u[e] >> 23) & 0xFFu) - emin, w);
      fz_put(s + pm, j * mb, (u[e] & 0x7FFFFFu) >> (23 - mb), mb);
    }
  }
  if (lane == 0) s[0] = emin | ((uint32_t)w << 8) | ((uint32_t)mb << 16);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint32_t* table = out32 + 4;
  uint32_t* dst = out32 + 4 + nblk + 1 + table[b];
  for (uint32_t q = lane; q < nw; q += 64) dst[q] = s[q];
}

__device__ __forceinline__ uint32_t fz_get(const uint32_t* __restrict__ p, uint32_t pos, int bits) {
  if (!bits) return 0u;
  const uint32_t wi = pos >> 5, sh = pos & 31u;
  uint64_t v = p[wi];
  if (sh + bits > 32) v |= (uint64_t)p[wi + 1] << 32;
  return (uint32_t)(v >> sh) & (bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u));
}

__global__ void __launch_bounds__(256) fz_decode_kernel(const uint32_t* __restrict__ in32,
                                                        int64_t nwords, int64_t n,
                                                        int64_t nblk, int prec, int mb,
                                                        float* __restrict__ out,
                                                        uint32_t* __restrict__ status) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nblk) return;
  const int lane = threadIdx.x & 63;
  const uint32_t* table = in32 + 4;
  const uint32_t off = table[b], end = table[b + 1];
  const int64_t area = nwords - (4 + nblk + 1);  // words available to the blocks
  const int64_t base = b * FZ_B;
  const int cnt = (int)((n - base) < FZ_B ? (n - base) : FZ_B);
  bool bad = in32[0] != FZ_MAGIC || in32[1] != (uint32_t)n || in32[2] != (uint32_t)prec ||
             in32[3] != (uint32_t)nblk || off >= end || (int64_t)end > area;
  uint32_t meta = 0;
  if (!bad) {
    meta = in32[4 + nblk + 1 + off];
    const int w0 = (int)((meta >> 8) & 0xFFu);
    bad = w0 > 8 || (int)((meta >> 16) & 0xFFu) != mb || end - off != fz_words(cnt, w0, mb) ||
          (meta >> 24) != 0u;
  }
  if (bad) {  // malformed stream: record it, write nothing
    if (lane == 0) atomicOr(status, 1u);
    return;
  }
  const uint32_t* blk = in32 + 4 + nblk + 1 + off;
  const uint32_t emin = meta & 0xFFu;
  const int w = (int)((meta >> 8) & 0xFFu);
  const uint32_t* ps = blk + 1;
  const uint32_t* pe = ps + (cnt + 31) / 32;
  const uint32_t* pm = pe + (cnt * w + 31) / 32;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t j = 4u * lane + e;
    uint32_t u = 0;
    if ((int)j < cnt) {
      u = (fz_get(ps, j, 1) << 31) | (((emin + fz_get(pe, j * w, w)) & 0xFFu) << 23) |
          (fz_get(pm, j * mb, mb) << (23 - mb));
    }
    v[e] = __uint_as_float(u);
  }
  const int64_t i0 = base + 4 * lane;
  if (4 * lane + 3 < cnt && aligned16(out)) {
    *reinterpret_cast<float4*>(out + i0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (4 * lane + e < cnt) out[i0 + e] = v[e];
  }
}

static inline size_t fz_al256(size_t v) { return (v + 255) & ~size_t(255); }

// stored precision (32 = lossless) and mantissa bits of a requested precision; -1 if invalid
static inline int fz_mbits(int precision, int* prec_out) {
  if (precision < 0) return -1;
  if (precision == 0 || precision >= 32) {
    *prec_out = 32;
    return 23;
  }
  *prec_out = precision;
  return precision > 9 ? precision - 9 : 0;
}

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_fpz_max_bytes(int64_t n) {
  if (n < 0) return 0;
  const int64_t nblk = (n + FZ_B - 1) / FZ_B;
  return 4 * (4 + nblk + 1 + nblk * (int64_t)FZ_MAXW);
}

extern "C" size_t dpz_fpz_workspace_bytes(int64_t n) {
  const int64_t nblk = n > 0 ? (n + FZ_B - 1) / FZ_B : 1;
  return fz_al256(sizeof(FzHdr)) + fz_al256((size_t)nblk * 4);
}

extern "C" int dpz_fpz_encode(const float* x, int64_t n, int precision, uint8_t* out,
                              int64_t out_cap, int64_t* nbytes_host, void* ws, size_t ws_bytes,
                              dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  int prec = 0;
  const int mb = fz_mbits(precision, &prec);
  if (mb < 0) return DPZ_ERR_UNSUPPORTED;
  if (n < 0 || n > FZ_MAXN || (n > 0 && !x) || !out || !nbytes_host) return DPZ_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(out) & 3u) || out_cap < dpz_fpz_max_bytes(n)) return DPZ_ERR_ARG;
  if (!ws || ws_bytes < dpz_fpz_workspace_bytes(n)) return DPZ_ERR_WORKSPACE;
  const int64_t nblk = (n + FZ_B - 1) / FZ_B;
  char* p = static_cast<char*>(ws);
  FzHdr* hdr = reinterpret_cast<FzHdr*>(p);
  uint32_t* blk_words = reinterpret_cast<uint32_t*>(p + fz_al256(sizeof(FzHdr)));
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  const unsigned grid = (unsigned)((nblk + 3) / 4);
  if (nblk > 0)
    DPZ_TIMED(DPZ_KT_FPZ_SIZE, st, fz_size_kernel<<<grid, 256, 0, st>>>(x, n, nblk, prec, mb, blk_words));
  DPZ_TIMED(DPZ_KT_FPZ_SCAN, st, fz_scan_kernel<<<1, 1024, 0, st>>>(n, nblk, prec, blk_words, out32, hdr));
  if (nblk > 0)
    DPZ_TIMED(DPZ_KT_FPZ_PACK, st, fz_pack_kernel<<<grid, 256, 0, st>>>(x, n, nblk, prec, mb, out32));
  FzHdr h;
  DPZ_HIP_TRY(hipMemcpyAsync(&h, hdr, sizeof(h), hipMemcpyDeviceToHost, st));
  DPZ_HIP_TRY(hipStreamSynchronize(st));
  *nbytes_host = (int64_t)h.nbytes;
  return DPZ_OK;
}

extern "C" int dpz_fpz_decode(const uint8_t* in, int64_t nbytes, int64_t n, int precision,
                              float* out, uint32_t* status, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  int prec = 0;
  const int mb = fz_mbits(precision, &prec);
  if (mb < 0) return DPZ_ERR_UNSUPPORTED;
  if (!in || n < 0 || n > FZ_MAXN || (n > 0 && !out) || !status) return DPZ_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(in) & 3u) || (nbytes & 3)) return DPZ_ERR_ARG;
  const int64_t nblk = (n + FZ_B - 1) / FZ_B;
  // the block area must at least hold the header, the table and one meta word a block
  if (nbytes < 4 * (4 + nblk + 1 + nblk)) return DPZ_ERR_ARG;
  if (nblk == 0) return DPZ_OK;
  const unsigned grid = (unsigned)((nblk + 3) / 4);
  DPZ_TIMED(DPZ_KT_FPZ_DECODE, st, fz_decode_kernel<<<grid, 256, 0, st>>>(
      reinterpret_cast<const uint32_t*>(in), nbytes / 4, n, nblk, prec, mb, out, status));
  return DPZ_OK;
}
