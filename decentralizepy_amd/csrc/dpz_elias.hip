// Elias-gamma coding of sorted index gaps, byte-compatible with the reference.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   compression/Elias.py:20-52  Elias.compress   (numpy, 15 ms at k = 110k)
//   compression/Elias.py:54-97  Elias.decompress (Python generator pointer chase, 316 ms at 110k)
//
// Format: first = a[0]; gaps g = diff(a) (uint32); l = floor(log2 g); every gap is written as l
// zero bits followed by g in l+1 bits MSB first; codes are concatenated; 128 zero bits follow;
// bytes are packed MSB-first (np.packbits); bytes [-16:-8] = int64 LE first, [-8:] = int64 LE
// total bit count (code bits + 128).
//
// Encode (3 launches): count (per-block code-bit totals) -> 1-block scan (block bit offsets, the
// zeroed padding / trailer words, zeroed block-boundary words) -> pack (each block assembles its
// codes into big-endian-bit 32-bit words in LDS; interior words are stored, the two boundary words
// shared with neighbouring blocks are OR-ed in).
// Decode (3 launches): speculate (one wave per 1024-bit chunk; lane o parses the chunk as if a
// code started at offset o, for every possible o < 63, recording exit offset, code count and gap
// sum) -> resolve (1 block: chain the chunks' true entry offsets through 64-chunk super maps, scan
// counts and gap sums) -> write (one wave per chunk re-parses its true path from LDS and writes
// first + running gap sums).
#include "dpz_common.h"

namespace dpz {

constexpr int EL_CODES = 1024;   // codes per encode block (4 per thread)
constexpr int EL_CHUNK = 1024;   // bits per decode chunk
constexpr int EL_CW = EL_CHUNK / 32;
constexpr int EL_STAGE = EL_CW + 4;  // staged words per chunk (a code may run 62 bits past)
constexpr int EL_SUPER = 64;     // chunks per super map
constexpr int EL_MAX_SUPER = 1024;  // => at most 2^26 code bits per stream

struct ElHdr {
  uint64_t L;       // code bits
  uint64_t nbits;   // L + 128
  uint64_t nbytes;  // ceil(nbits / 8)
  uint32_t status;  // 0 ok, 1 invalid input
  uint32_t pad;
  uint64_t count;   // decode: number of values (codes + 1)
};

__device__ __forceinline__ uint32_t code_len(uint32_t g) { return 2u * (31u - __clz(g)) + 1u; }

// ---------------------------------------------------------------- encode
__global__ void __launch_bounds__(256) elias_count_kernel(const int32_t* __restrict__ idx,
                                                          int64_t ncodes, uint64_t* blk_bits,
                                                          ElHdr* hdr) {
  __shared__ uint64_t wsum[16];
  const int64_t base = (int64_t)blockIdx.x * EL_CODES + threadIdx.x * 4;
  uint64_t bits = 0;
  bool bad = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = base + e;
    if (i < ncodes) {
      const uint32_t g = (uint32_t)(idx[i + 1] - idx[i]);
      if (g == 0 || (int32_t)g < 0) bad = true;
      bits += g ? code_len(g) : 1u;
    }
  }
  if (bad) hdr->status = 1;
  uint64_t tot;
  block_excl_scan64(bits, wsum, &tot);
  if (threadIdx.x == 0) blk_bits[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) elias_scan_kernel(const int32_t* __restrict__ idx,
                                                          int64_t nblk, const uint64_t* blk_bits,
                                                          uint64_t* blk_off, ElHdr* hdr,
                                                          uint32_t* out32) {
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t s_L;
  uint64_t carry = 0;
  for (int64_t b0 = 0; b0 < nblk; b0 += 1024) {
    const int64_t b = b0 + threadIdx.x;
    const uint64_t v = b < nblk ? blk_bits[b] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot) + carry;
    if (b < nblk) blk_off[b] = ex;
    carry += tot;
  }
  if (threadIdx.x == 0) s_L = carry;
  __syncthreads();
  const uint64_t L = s_L;
  const uint64_t nbits = L + 128;
  const uint64_t nbytes = (nbits + 7) >> 3;
  const uint64_t tail_w0 = L >> 5;
  const uint64_t nwords = (nbytes + 3) >> 2;
  // zero the boundary words below the tail (they are OR-ed by the pack kernel)
  for (int64_t b = threadIdx.x; b < nblk; b += 1024) {
    const uint64_t o = blk_off[b], n = blk_bits[b];
    const uint64_t wf = o >> 5, wl = (o + n - 1) >> 5;
    if (wf < tail_w0) out32[wf] = 0u;
    if (wl < tail_w0) out32[wl] = 0u;
  }
  // tail words: zero padding + trailer (int64 LE first, int64 LE nbits) in byte order
  const uint64_t first = (uint64_t)(int64_t)idx[0];
  for (uint64_t w = tail_w0 + threadIdx.x; w < nwords; w += 1024) {
    uint32_t val = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t B = 4 * w + j;
      uint32_t byte = 0;
      if (B >= nbytes - 16 && B < nbytes - 8) byte = (uint32_t)(first >> (8 * (B - (nbytes - 16)))) & 0xFFu;
      else if (B >= nbytes - 8 && B < nbytes) byte = (uint32_t)(nbits >> (8 * (B - (nbytes - 8)))) & 0xFFu;
      val |= byte << (8 * j);
    }
    out32[w] = val;
  }
  if (threadIdx.x == 0) {
    hdr->L = L;
    hdr->nbits = nbits;
    hdr->nbytes = nbytes;
  }
}

__global__ void __launch_bounds__(256) elias_pack_kernel(const int32_t* __restrict__ idx,
                                                         int64_t ncodes,
                                                         const uint64_t* __restrict__ blk_bits,
                                                         const uint64_t* __restrict__ blk_off,
                                                         uint32_t* out32) {
  constexpr int MAXW = (EL_CODES * 63 + 31) / 32 + 2;
  __shared__ uint32_t words[MAXW];
  __shared__ uint64_t wsum[16];
  const uint64_t B0 = blk_off[blockIdx.x];
  const uint64_t B1 = B0 + blk_bits[blockIdx.x];
  const uint64_t w0 = B0 >> 5, w1 = (B1 - 1) >> 5;
  const int nw = (int)(w1 - w0 + 1);
  for (int w = threadIdx.x; w < nw; w += 256) words[w] = 0u;
  const int64_t base = (int64_t)blockIdx.x * EL_CODES + threadIdx.x * 4;
  uint32_t g[4], len[4];
  uint64_t mine = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = base + e;
    g[e] = 0;
    len[e] = 0;
    if (i < ncodes) {
      g[e] = (uint32_t)(idx[i + 1] - idx[i]);
      len[e] = g[e] ? code_len(g[e]) : 1u;
    }
    mine += len[e];
  }
  uint64_t tot;
  uint64_t off = block_excl_scan64(mine, wsum, &tot) + B0;  // contains barriers (words zeroed)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (len[e] > 1 || (len[e] == 1 && g[e])) {
      const uint32_t l = (len[e] - 1) >> 1;
      const uint32_t n = l + 1;
      const uint64_t rel = off + l - 32 * w0;  // value bits start here
      const int wi = (int)(rel >> 5);
      const uint32_t b = (uint32_t)(rel & 31);
      const uint64_t v64 = (uint64_t)g[e] << (64 - b - n);
      const uint32_t hi = (uint32_t)(v64 >> 32), lo = (uint32_t)v64;
      if (hi) atomicOr(&words[wi], hi);
      if (lo) atomicOr(&words[wi + 1], lo);
    }
    off += len[e];
  }
  __syncthreads();
  for (int w = threadIdx.x; w < nw; w += 256) {
    const uint32_t val = __builtin_bswap32(words[w]);
    if (w == 0 || w == nw - 1) {
      if (val) atomicOr(&out32[w0 + w], val);
    } else {
      out32[w0 + w] = val;
    }
  }
}

// ---------------------------------------------------------------- decode
__device__ __forceinline__ uint64_t window64(const uint32_t* words, uint64_t rel) {
  const int wi = (int)(rel >> 5);
  const uint32_t sh = (uint32_t)(rel & 31);
  const uint64_t a = ((uint64_t)words[wi] << 32) | words[wi + 1];
  return sh ? ((a << sh) | (words[wi + 2] >> (32 - sh))) : a;
}

// wave per chunk: lane o parses from chunk_start + o
__global__ void __launch_bounds__(256) elias_spec_kernel(const uint32_t* __restrict__ in32,
                                                         uint64_t nwords_in, uint64_t L,
                                                         int64_t nch, uint8_t* exit_tab,
                                                         uint32_t* cnt_tab, uint64_t* sum_tab) {
  __shared__ uint32_t st[4][EL_STAGE];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + wid;
  const uint64_t wbase = (uint64_t)c * EL_CW;
  if (lane < EL_STAGE) {
    const uint64_t w = wbase + lane;
    st[wid][lane] = w < nwords_in ? __builtin_bswap32(in32[w]) : 0u;
  }
  __syncthreads();
  if (c >= nch) return;
  const uint64_t cstart = (uint64_t)c * EL_CHUNK;
  const uint64_t cend = (cstart + EL_CHUNK < L) ? cstart + EL_CHUNK : L;
  uint64_t pos = cstart + lane;
  uint32_t cnt = 0;
  uint64_t gsum = 0;
  uint8_t ex = 0xFF;
  if (lane < 63 && pos < cend) {
    bool ok = true;
    while (pos < cend) {
      const uint64_t w = window64(st[wid], pos - wbase * 32);
      const uint32_t z = (uint32_t)__clzll((long long)w);
      if (w == 0 || z > 31) { ok = false; break; }
      const uint32_t n = z + 1;
      const uint64_t gv = (w << z) >> (64 - n);
      gsum += gv;
      ++cnt;
      pos += 2 * z + 1;
    }
    if (ok) ex = (uint8_t)(pos - cend);  // < 63
  } else if (lane < 63 && pos >= cend) {
    ex = (uint8_t)(pos - cend);  // entry beyond this (last) chunk's end
  }
  exit_tab[c * 64 + lane] = ex;
  cnt_tab[c * 64 + lane] = cnt;
  sum_tab[c * 64 + lane] = gsum;
}

__global__ void __launch_bounds__(1024) elias_resolve_kernel(int64_t nch,
                                                             const uint8_t* __restrict__ exit_tab,
                                                             const uint32_t* __restrict__ cnt_tab,
                                                             const uint64_t* __restrict__ sum_tab,
                                                             uint32_t* chunk_entry,
                                                             uint64_t* chunk_pos,
                                                             uint64_t* chunk_base, ElHdr* hdr) {
  __shared__ uint8_t sexit[EL_MAX_SUPER][64];        // super maps (64 KB)
  __shared__ uint32_t stab[16][EL_SUPER * 64 / 4];  // per-wave staged chunk maps (64 KB)
  __shared__ uint8_t sent[16][EL_SUPER];
  __shared__ uint16_t sentry[EL_MAX_SUPER + 1];
  __shared__ uint64_t wsum[16];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t S = (nch + EL_SUPER - 1) / EL_SUPER;
  const uint8_t* tab = reinterpret_cast<const uint8_t*>(stab[wid]);
  auto stage = [&](int64_t s) {  // the chunk maps of super-chunk s -> this wave's LDS slot
    const int64_t c0 = s * EL_SUPER;
    const int64_t nc = (nch - c0) < EL_SUPER ? (nch - c0) : EL_SUPER;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(exit_tab + c0 * 64);
    for (int w = lane; w < nc * 16; w += 64) stab[wid][w] = src[w];
    return (int)nc;
  };
  // a) super maps: lane o walks the chunk maps of super-chunk s from entry o
  for (int64_t s0 = 0; s0 < S; s0 += 16) {
    const int64_t s = s0 + wid;
    int nc = 0;
    if (s < S) nc = stage(s);
    __syncthreads();
    if (s < S) {
      uint32_t e = lane < 63 ? lane : 0xFF;
      for (int j = 0; j < nc && e < 63; ++j) e = tab[j * 64 + e];
      sexit[s][lane] = (uint8_t)(e < 63 ? e : 0xFF);
    }
    __syncthreads();
  }
  // b) chain the super maps from entry 0
  if (threadIdx.x == 0) {
    uint32_t e = 0;
    for (int64_t s = 0; s < S; ++s) {
      sentry[s] = (uint16_t)e;
      e = (e < 63) ? sexit[s][e] : 0xFF;
    }
    sentry[S] = (uint16_t)e;
    if (e != 0) hdr->status = 1;  // the true path must end exactly at L
  }
  __syncthreads();
  // c) per-chunk true entries (lane 0 walks), then counts and gap sums (all lanes)
  for (int64_t s0 = 0; s0 < S; s0 += 16) {
    const int64_t s = s0 + wid;
    int nc = 0;
    if (s < S) nc = stage(s);
    __syncthreads();
    if (s < S && lane == 0) {
      uint32_t e = sentry[s];
      for (int j = 0; j < nc; ++j) {
        sent[wid][j] = (uint8_t)e;
        e = (e < 63) ? tab[j * 64 + e] : 0xFF;
      }
    }
    __syncthreads();
    if (s < S && lane < nc) {
      const int64_t c = s * EL_SUPER + lane;
      const uint32_t e = sent[wid][lane];
      chunk_entry[c] = e;
      if (e < 63) {
        chunk_pos[c] = cnt_tab[c * 64 + e];
        chunk_base[c] = sum_tab[c * 64 + e];
      } else {
        chunk_pos[c] = 0;
        chunk_base[c] = 0;
        hdr->status = 1;
      }
    }
    __syncthreads();
  }
  // d) exclusive scans of counts and gap sums over chunks (in place)
  uint64_t carry_n = 0, carry_s = 0;
  for (int64_t c0 = 0; c0 < nch; c0 += 1024) {
    const int64_t c = c0 + threadIdx.x;
    const uint64_t n = c < nch ? chunk_pos[c] : 0;
    const uint64_t sm = c < nch ? chunk_base[c] : 0;
    uint64_t tn, ts;
    const uint64_t pn = block_excl_scan64(n, wsum, &tn) + carry_n;
    const uint64_t ps = block_excl_scan64(sm, wsum, &ts) + carry_s;
    if (c < nch) {
      chunk_pos[c] = pn;
      chunk_base[c] = ps;
    }
    carry_n += tn;
    carry_s += ts;
  }
  if (threadIdx.x == 0) hdr->count = carry_n + 1;
}

// wave per chunk: lane 0 re-parses the true path from LDS and writes first + running sums
__global__ void __launch_bounds__(256) elias_write_kernel(const uint32_t* __restrict__ in32,
                                                          uint64_t nwords_in, uint64_t L,
                                                          int64_t nch, int64_t first,
                                                          const uint32_t* __restrict__ chunk_entry,
                                                          const uint64_t* __restrict__ chunk_pos,
                                                          const uint64_t* __restrict__ chunk_base,
                                                          const ElHdr* hdr, int64_t cap,
                                                          int64_t* out64, int32_t* out32) {
  __shared__ uint32_t st[4][EL_STAGE];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + wid;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (out64) out64[0] = first;
    if (out32) out32[0] = (int32_t)first;
  }
  const uint64_t wbase = (uint64_t)c * EL_CW;
  if (lane < EL_STAGE) {
    const uint64_t w = wbase + lane;
    st[wid][lane] = w < nwords_in ? __builtin_bswap32(in32[w]) : 0u;
  }
  __syncthreads();
  if (c >= nch || hdr->status || lane != 0) return;
  const uint64_t cstart = (uint64_t)c * EL_CHUNK;
  const uint64_t cend = (cstart + EL_CHUNK < L) ? cstart + EL_CHUNK : L;
  uint64_t pos = cstart + chunk_entry[c];
  int64_t o = 1 + (int64_t)chunk_pos[c];
  int64_t v = first + (int64_t)chunk_base[c];
  while (pos < cend) {
    const uint64_t w = window64(st[wid], pos - wbase * 32);
    const uint32_t z = (uint32_t)__clzll((long long)w);
    const uint32_t n = z + 1;
    v += (int64_t)((w << z) >> (64 - n));
    if (o < cap) {
      if (out64) out64[o] = v;
      if (out32) out32[o] = (int32_t)v;
    }
    ++o;
    pos += 2 * z + 1;
  }
}

struct ElEncWs {
  uint64_t* blk_bits;
  uint64_t* blk_off;
  ElHdr* hdr;
};

static inline size_t al256(size_t v) { return (v + 255) & ~size_t(255); }

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_elias_max_bytes(int64_t k) {
  if (k < 2) return 0;
  const int64_t bits = 63 * (k - 1) + 128;
  return ((bits + 31) / 32) * 4 + 16;
}

extern "C" size_t dpz_elias_workspace_bytes(int64_t k, int64_t nbytes) {
  const int64_t ncodes = k > 1 ? k - 1 : 1;
  const int64_t nblk = (ncodes + EL_CODES - 1) / EL_CODES;
  const int64_t nch = (nbytes * 8 + EL_CHUNK - 1) / EL_CHUNK + 1;
  const size_t enc = al256(sizeof(ElHdr)) + 2 * al256(nblk * 8);
  const size_t dec = al256(sizeof(ElHdr)) + al256(nch * 64) + al256(nch * 64 * 4) +
                     al256(nch * 64 * 8) + al256(nch * 4) + 2 * al256(nch * 8);
  return enc > dec ? enc : dec;
}

extern "C" int dpz_elias_encode(const int32_t* idx, int64_t k, uint8_t* out, int64_t out_cap,
                                int64_t* nbytes_host, void* ws, size_t ws_bytes,
                                dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (k < 2 || !idx || !out || !nbytes_host) return DPZ_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(out) & 3u) || out_cap < dpz_elias_max_bytes(k)) return DPZ_ERR_ARG;
  if (!ws || ws_bytes < dpz_elias_workspace_bytes(k, 0)) return DPZ_ERR_WORKSPACE;
  const int64_t ncodes = k - 1;
  const int64_t nblk = (ncodes + EL_CODES - 1) / EL_CODES;
  char* p = static_cast<char*>(ws);
  ElHdr* hdr = reinterpret_cast<ElHdr*>(p);
  uint64_t* blk_bits = reinterpret_cast<uint64_t*>(p + al256(sizeof(ElHdr)));
  uint64_t* blk_off = reinterpret_cast<uint64_t*>(p + al256(sizeof(ElHdr)) + al256(nblk * 8));
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  DPZ_HIP_TRY(hipMemsetAsync(hdr, 0, sizeof(ElHdr), st));
  DPZ_TIMED(DPZ_KT_ELIAS_COUNT, st, elias_count_kernel<<<(unsigned)nblk, 256, 0, st>>>(idx, ncodes, blk_bits, hdr));
  DPZ_TIMED(DPZ_KT_ELIAS_SCAN, st, elias_scan_kernel<<<1, 1024, 0, st>>>(idx, nblk, blk_bits, blk_off, hdr, out32));
  DPZ_TIMED(DPZ_KT_ELIAS_PACK, st, elias_pack_kernel<<<(unsigned)nblk, 256, 0, st>>>(idx, ncodes, blk_bits, blk_off, out32));
  ElHdr h;
  DPZ_HIP_TRY(hipMemcpyAsync(&h, hdr, sizeof(h), hipMemcpyDeviceToHost, st));
  DPZ_HIP_TRY(hipStreamSynchronize(st));
  if (h.status) return DPZ_ERR_ARG;  // unsorted or duplicate indices
  *nbytes_host = (int64_t)h.nbytes;
  return DPZ_OK;
}

namespace {

// The async decode's tail: the stream must hold exactly `count` values (the caller knows the
// count from the payload's other leg), else the status word is OR-ed nonzero.
__global__ void elias_check_kernel(const ElHdr* hdr, int64_t count, uint32_t* status) {
  if (threadIdx.x == 0 && (hdr->status || (int64_t)hdr->count != count)) atomicOr(status, 1u);
}

// a one-value stream (L == 0), written on the device (no host source for an async copy)
__global__ void elias_single_kernel(int64_t first, int64_t count, int64_t* out64, int32_t* out32,
                                    uint32_t* status) {
  if (threadIdx.x != 0) return;
  if (out64) out64[0] = first;
  if (out32) out32[0] = (int32_t)first;
  if (status && count != 1) atomicOr(status, 1u);
}

// argument checks + the three decode launches; *hdr_out = the header the launches fill
int elias_decode_launch(const uint8_t* in, int64_t nbytes, int64_t nbits, int64_t first,
                        int64_t* out64, int32_t* out32, int64_t out_cap, void* ws,
                        size_t ws_bytes, hipStream_t st, ElHdr** hdr_out) {
  if (!in || nbytes < 16 || nbits < 128 || (!out64 && !out32)) return DPZ_ERR_ARG;
  if (reinterpret_cast<uintptr_t>(in) & 3u) return DPZ_ERR_ARG;
  const uint64_t L = (uint64_t)(nbits - 128);
  if ((uint64_t)nbytes * 8 < L) return DPZ_ERR_ARG;
  const int64_t nch = (int64_t)((L + EL_CHUNK - 1) / EL_CHUNK);
  if ((nch + EL_SUPER - 1) / EL_SUPER > EL_MAX_SUPER) return DPZ_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < dpz_elias_workspace_bytes(2, nbytes)) return DPZ_ERR_WORKSPACE;
  *hdr_out = nullptr;
  if (L == 0) return DPZ_OK;
  char* p = static_cast<char*>(ws);
  size_t o = 0;
  ElHdr* hdr = reinterpret_cast<ElHdr*>(p + o); o += al256(sizeof(ElHdr));
  uint8_t* exit_tab = reinterpret_cast<uint8_t*>(p + o); o += al256(nch * 64);
  uint32_t* cnt_tab = reinterpret_cast<uint32_t*>(p + o); o += al256(nch * 64 * 4);
  uint64_t* sum_tab = reinterpret_cast<uint64_t*>(p + o); o += al256(nch * 64 * 8);
  uint32_t* centry = reinterpret_cast<uint32_t*>(p + o); o += al256(nch * 4);
  uint64_t* cpos = reinterpret_cast<uint64_t*>(p + o); o += al256(nch * 8);
  uint64_t* cbase = reinterpret_cast<uint64_t*>(p + o); o += al256(nch * 8);
  const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
  const uint64_t nwords_in = (uint64_t)(nbytes - 16 + 3) / 4;  // code + padding words (trailer excluded)
  DPZ_HIP_TRY(hipMemsetAsync(hdr, 0, sizeof(ElHdr), st));
  const unsigned grid = (unsigned)((nch + 3) / 4);
  DPZ_TIMED(DPZ_KT_ELIAS_SPEC, st, elias_spec_kernel<<<grid, 256, 0, st>>>(in32, nwords_in, L, nch, exit_tab, cnt_tab, sum_tab));
  DPZ_TIMED(DPZ_KT_ELIAS_RESOLVE, st, elias_resolve_kernel<<<1, 1024, 0, st>>>(nch, exit_tab, cnt_tab, sum_tab, centry, cpos, cbase, hdr));
  DPZ_TIMED(DPZ_KT_ELIAS_WRITE, st, elias_write_kernel<<<grid, 256, 0, st>>>(in32, nwords_in, L, nch, first, centry, cpos, cbase, hdr,
                                           out_cap, out64, out32));
  *hdr_out = hdr;
  return DPZ_OK;
}

}  // namespace

extern "C" int dpz_elias_decode(const uint8_t* in, int64_t nbytes, int64_t nbits, int64_t first,
                                int64_t* out64, int32_t* out32, int64_t out_cap,
                                int64_t* count_host, void* ws, size_t ws_bytes,
                                dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!count_host) return DPZ_ERR_ARG;
  ElHdr* hdr = nullptr;
  const int rc = elias_decode_launch(in, nbytes, nbits, first, out64, out32, out_cap, ws, ws_bytes,
                                     st, &hdr);
  if (rc != DPZ_OK) return rc;
  if (!hdr) {  // a single value (the reference cannot produce it, but decode it consistently)
    *count_host = 1;
    if (out_cap >= 1) {
      elias_single_kernel<<<1, 64, 0, st>>>(first, 1, out64, out32, nullptr);
      DPZ_HIP_TRY(hipStreamSynchronize(st));
    }
    return DPZ_OK;
  }
  ElHdr h;
  DPZ_HIP_TRY(hipMemcpyAsync(&h, hdr, sizeof(h), hipMemcpyDeviceToHost, st));
  DPZ_HIP_TRY(hipStreamSynchronize(st));
  if (h.status) return DPZ_ERR_ARG;  // malformed stream
  *count_host = (int64_t)h.count;
  if ((int64_t)h.count > out_cap) return DPZ_ERR_WORKSPACE;
  return DPZ_OK;
}

extern "C" int dpz_elias_decode_async(const uint8_t* in, int64_t nbytes, int64_t nbits,
                                      int64_t first, int64_t* out64, int32_t* out32, int64_t count,
                                      uint32_t* status, void* ws, size_t ws_bytes,
                                      dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!status || count < 1) return DPZ_ERR_ARG;
  ElHdr* hdr = nullptr;
  const int rc = elias_decode_launch(in, nbytes, nbits, first, out64, out32, count, ws, ws_bytes,
                                     st, &hdr);
  if (rc != DPZ_OK) return rc;
  if (!hdr) {
    elias_single_kernel<<<1, 64, 0, st>>>(first, count, out64, out32, status);
  } else {
    elias_check_kernel<<<1, 64, 0, st>>>(hdr, count, status);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DPZ_OK : (int)e;
}
