// LZ4 frame codec on the device: the wire format of the reference's Lz4Wrapper compressor.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   compression/Lz4Wrapper.py:20-41   lz4.frame.compress(np.diff(sorted idx).tobytes())
//   compression/Lz4Wrapper.py:43-61   np.cumsum(np.frombuffer(lz4.frame.decompress(b), int32))
//   compression/Lz4Wrapper.py:63-98   the same frame codec on the fp32 value bytes
// (python-lz4's lz4.frame, third-party, absent here; its frame format is the LZ4 frame spec and
// its default preferences are: 64 KB blocks, linked, content size stored, no checksums).
//
// Encoder: the input is cut into 2 KB blocks (DPZ_LZ_BLK), ONE WAVE per block; the frame is
// LINKED (B.Indep clear, python-lz4's default mode): a block's matches may reach DPZ_LZ_WIN
// (14 KB) back into the input before it, which every block reads from the input itself, so the
// blocks are still encoded in parallel:
//   1. the history and the block are staged in LDS; the hash table (LZ4's 5-byte multiplicative
//      hash, 12 bits) is prefilled with the history's positions, then every position
//      i <= len - 12 of the block hashes its 5 bytes 64 positions at a time: the candidate is the
//      table entry left by earlier chunks, then the chunk publishes itself with LDS atomicMax
//      (the nearest earlier occurrence wins — deterministic);
//   2. each lane extends its candidate word-wise (min match 4, capped at 1024 and at len - 5) and
//      sets its bit in a per-position match mask;
//   3. the greedy parse walks the mask with 64-bit bit scans (literal runs cost one scan, not one
//      step per byte) and records the sequences in LDS;
//   4. sequence sizes, a wave scan, and every lane emits its sequences into an LDS output buffer,
//      copied out coalesced; a block that does not shrink is stored uncompressed (LZ4 frame
//      high-bit block size).
// A second launch scans the block sizes and assembles the frame (header, size-prefixed blocks,
// end mark).  Decoder: the host walks the frame's block headers (it holds the bytes).  Blocks
// that decode to <= 4 KB take the parallel decoder — every block parsed from all byte positions
// at once, each output byte given its source (a literal, an earlier byte of the block, or for a
// linked frame an earlier block's byte), pointer jumping inside the block; then the blocks are
// placed at their frame offsets and references into earlier blocks are resolved by pointer
// jumping over the whole frame (lz4_link_place_kernel, lz4_link_resolve_kernel).  liblz4's 64 KB
// linked blocks decode in ONE workgroup block after block with a 64 KB LDS ring window.  Every
// read / write is bounds-checked; a malformed block sets *status.
#include "dpz_common.h"

namespace dpz {

#ifndef DPZ_LZ_BLK
#define DPZ_LZ_BLK 2048
#endif
#ifndef DPZ_LZ_HASH_LOG
#define DPZ_LZ_HASH_LOG 12
#endif
// history a block's matches may reach back into (the previous blocks' input): the frame is
// LINKED (B.Indep = 0, python-lz4's default block mode).  0: independent blocks.
#ifndef DPZ_LZ_WIN
#define DPZ_LZ_WIN 14336
#endif
constexpr int LZ_BLK = DPZ_LZ_BLK;  // encoder block (one wave)
constexpr int LZ_HASH_LOG = DPZ_LZ_HASH_LOG;
constexpr int LZ_WIN = DPZ_LZ_WIN;
static_assert(LZ_WIN % 64 == 0 && LZ_WIN + LZ_BLK < 65536, "window + block inside LZ4's 64 KB");
static_assert(LZ_BLK >= 256 && LZ_BLK <= 65536 && (LZ_BLK & 63) == 0, "encoder block size");
constexpr int LZ_MAXM = 1024;       // match length cap
constexpr int LZ_MFLIMIT = 12;      // a match starts at least 12 bytes before the block end
constexpr int LZ_LASTLIT = 5;       // the last 5 bytes are literals
constexpr int LZ_BLK_OUT = LZ_BLK + 64;  // per-block encoder output slot (raw fallback fits)
constexpr int LZ_MAXSEQ = LZ_BLK / 4;
constexpr uint32_t LZ_MAGIC = 0x184D2204u;
constexpr int LZ_HDR = 15;          // magic 4 + FLG + BD + content size 8 + HC

// ---- encoder --------------------------------------------------------------------------------
struct LzEncLds {
  uint32_t data[(LZ_WIN + LZ_BLK) / 4 + 2];  // history + the block (+8 zero bytes of slack)
  uint32_t table[1 << LZ_HASH_LOG];   // position + 1 of the latest occurrence (0 = none)
  uint32_t minfo[LZ_BLK];             // (match length << 16) | offset, per position
  unsigned long long mask[LZ_BLK / 64];
  uint2 seq[LZ_MAXSEQ + 1];           // (literal start | literal length << 16, offset | ml << 16)
  uint32_t nseq;
};

__device__ __forceinline__ uint32_t lz_read32(const uint32_t* w, int i) {
  const int q = i >> 2, r = i & 3;
  if (r == 0) return w[q];
  return (w[q] >> (8 * r)) | (w[q + 1] << (32 - 8 * r));
}

__device__ __forceinline__ uint32_t lz_byte(const uint32_t* w, int i) {
  return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
}

__device__ __forceinline__ int lz_lenext(int L) { return L >= 15 ? (L - 15) / 255 + 1 : 0; }

__device__ __forceinline__ void lz_put(uint8_t* ob, int pos, uint32_t v) { ob[pos] = (uint8_t)v; }

// Global bytes -> LDS, one wave: every load of a round issued before its LDS writes (a loop of
// load -> wait -> write per byte is one memory round trip per 64 bytes).  16-byte loads when the
// source is aligned, else 16 independent byte loads per lane per round.
// (No local arrays: indexed temporaries were placed in scratch memory — 80 bytes per lane, a
// global round trip per staged word; vector-typed temporaries stay in registers.)
__device__ __forceinline__ void lz_stage(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t n) {
  const int lane = threadIdx.x & 63;
  if ((reinterpret_cast<uintptr_t>(src) & 15u) == 0) {
    const uint32_t nv = n / 16;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (uint32_t v0 = 0; v0 < nv; v0 += 4 * 64) {  // loads branch-free (indices clamped)
      const uint32_t v = v0 + lane, last = nv - 1;
      const uint4 r0 = s4[v < nv ? v : last];
      const uint4 r1 = s4[v + 64 < nv ? v + 64 : last];
      const uint4 r2 = s4[v + 128 < nv ? v + 128 : last];
      const uint4 r3 = s4[v + 192 < nv ? v + 192 : last];
      if (v < nv) d4[v] = r0;
      if (v + 64 < nv) d4[v + 64] = r1;
      if (v + 128 < nv) d4[v + 128] = r2;
      if (v + 192 < nv) d4[v + 192] = r3;
    }
    for (uint32_t t = nv * 16 + lane; t < n; t += 64) dst[t] = src[t];
    return;
  }
  // unaligned source: 16 independent byte loads per lane per round, packed into four words
  for (uint32_t t0 = 0; t0 < n; t0 += 16 * 64) {
#define DPZ_LZB(u) ((t0 + (u) * 64u + lane) < n ? (uint32_t)src[t0 + (u) * 64u + lane] : 0u)
    const uint32_t w0 = DPZ_LZB(0) | DPZ_LZB(1) << 8 | DPZ_LZB(2) << 16 | DPZ_LZB(3) << 24;
    const uint32_t w1 = DPZ_LZB(4) | DPZ_LZB(5) << 8 | DPZ_LZB(6) << 16 | DPZ_LZB(7) << 24;
    const uint32_t w2 = DPZ_LZB(8) | DPZ_LZB(9) << 8 | DPZ_LZB(10) << 16 | DPZ_LZB(11) << 24;
    const uint32_t w3 = DPZ_LZB(12) | DPZ_LZB(13) << 8 | DPZ_LZB(14) << 16 | DPZ_LZB(15) << 24;
#undef DPZ_LZB
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint32_t t = t0 + u * 64 + lane;
      const uint32_t w = u < 4 ? w0 : (u < 8 ? w1 : (u < 12 ? w2 : w3));
      if (t < n) dst[t] = (uint8_t)(w >> (8 * (u & 3)));
    }
  }
}

// one wave per 4 KB block; blocks of 64 threads
__global__ void __launch_bounds__(64) lz4_encode_blocks(const uint8_t* __restrict__ in, int64_t n,
                                                       uint8_t* __restrict__ slots,
                                                       uint32_t* __restrict__ bsize) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lz_smem[];
  LzEncLds& S = *reinterpret_cast<LzEncLds*>(lz_smem);
  const int lane = threadIdx.x;
  const int64_t blk = blockIdx.x;
  const int64_t base = blk * LZ_BLK;
  const int len = (int)((n - base) < LZ_BLK ? (n - base) : LZ_BLK);
  // LDS holds [base - hist, base + len): the history the block's matches may reach (linked
  // frame) and the block; every position below is an LDS position (the block starts at hist)
  const int hist = (int)(base < LZ_WIN ? base : LZ_WIN);
  for (int w = lane; w < (LZ_WIN + LZ_BLK) / 4 + 2; w += 64) S.data[w] = 0;
  __syncthreads();
  lz_stage(reinterpret_cast<uint8_t*>(S.data), in + base - hist, (uint32_t)(hist + len));
  for (int t = lane; t < (1 << LZ_HASH_LOG); t += 64) S.table[t] = 0;
  for (int t = lane; t < LZ_BLK / 64; t += 64) S.mask[t] = 0ull;
  __syncthreads();
  // 5-byte hash (LZ4's hash5 for 64-bit targets): a candidate that agrees in 5 bytes usually
  // extends past 4 — on index gaps ("yy 00 00 00" words) 4-byte-hash candidates give 4-5 byte
  // matches that barely pay for their token, 5-byte ones the longer runs liblz4 finds
  auto hash5 = [&](int i) {
    const uint64_t v = (uint64_t)lz_read32(S.data, i) | ((uint64_t)lz_read32(S.data, i + 4) << 32);
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - LZ_HASH_LOG));
  };
  // the history's positions into the table, in order (the latest occurrence wins)
  for (int c0 = 0; c0 < hist; c0 += 64) {
    const int i = c0 + lane;
    const uint32_t h = hash5(i);
    if (i < hist) atomicMax(&S.table[h], (uint32_t)(i + 1));
    __syncthreads();
  }
  const int last_start = hist + len - LZ_MFLIMIT;  // match starts i <= last_start
  const int mend = hist + len - LZ_LASTLIT;        // a match ends at or before mend
  for (int c0 = hist; c0 <= last_start; c0 += 64) {
    const int i = c0 + lane;
    const bool ok = i <= last_start;
    uint32_t v = 0, h = 0, cand = 0;
    if (ok) {
      v = lz_read32(S.data, i);
      h = hash5(i);
      cand = S.table[h];
    }
    __syncthreads();
    if (ok) atomicMax(&S.table[h], (uint32_t)(i + 1));
    uint32_t info = 0;
    if (ok && cand != 0) {
      const int j = (int)cand - 1;
      if (lz_read32(S.data, j) == v) {
        int ml = 4;
        const int cap = (mend - i) < LZ_MAXM ? (mend - i) : LZ_MAXM;
        while (ml + 4 <= cap) {
          const uint32_t x = lz_read32(S.data, i + ml) ^ lz_read32(S.data, j + ml);
          if (x) {
            ml += __builtin_ctz(x) >> 3;
            break;
          }
          ml += 4;
        }
        if (ml + 4 > cap) {  // byte tail (or the capped word loop ran out)
          while (ml < cap && lz_byte(S.data, i + ml) == lz_byte(S.data, j + ml)) ++ml;
        }
        if (ml > cap) ml = cap;
        if (ml >= 4) info = ((uint32_t)ml << 16) | (uint32_t)(i - j);
      }
    }
    if (ok) S.minfo[i - hist] = info;
    const unsigned long long bal = __ballot(info != 0);
    if (lane == 0) S.mask[(c0 - hist) >> 6] = bal;
    __syncthreads();
  }
  __syncthreads();
  // greedy parse (wave-uniform): jump from match end to the next match start by bit scans (the
  // mask and minfo are indexed from the block start; p, q, lit are LDS positions)
  uint32_t nseq = 0;
  int p = hist, lit = hist;
  for (;;) {
    int q = -1;
    if (p <= last_start) {
      int wi = (p - hist) >> 6;
      unsigned long long w = S.mask[wi] & (~0ull << ((p - hist) & 63));
      const int wlast = (last_start - hist) >> 6;
      while (w == 0ull && wi < wlast) w = S.mask[++wi];
      if (w != 0ull) q = hist + (wi << 6) + __builtin_ctzll(w);
    }
    if (q < 0) break;
    const uint32_t info = S.minfo[q - hist];
    const int ml = (int)(info >> 16), off = (int)(info & 0xFFFFu);
    if (lane == 0)
      S.seq[nseq] = make_uint2((uint32_t)lit | ((uint32_t)(q - lit) << 16),
                               (uint32_t)off | ((uint32_t)ml << 16));
    ++nseq;
    p = q + ml;
    lit = p;
  }
  // the last sequence: literals only
  if (lane == 0) S.seq[nseq] = make_uint2((uint32_t)lit | ((uint32_t)(hist + len - lit) << 16), 0u);
  __syncthreads();
  const uint32_t ns = nseq + 1;
  // sizes and offsets of the sequences (wave scan in chunks of 64)
  uint8_t* ob = reinterpret_cast<uint8_t*>(S.minfo);  // reuse: 4 LZ_BLK bytes >= LZ_BLK_OUT
  uint32_t run = 0;
  for (uint32_t s0 = 0; s0 < ns; s0 += 64) {
    const uint32_t s = s0 + lane;
    int sz = 0;
    uint2 e = make_uint2(0, 0);
    if (s < ns) {
      e = S.seq[s];
      const int L = (int)(e.x >> 16);
      sz = 1 + lz_lenext(L) + L;
      if (s + 1 < ns) sz += 2 + lz_lenext((int)(e.y >> 16) - 4);
    }
    uint32_t tot;
    const uint32_t ex = wave_excl_scan((uint32_t)sz, &tot);
    if (s < ns) {
      int pos = (int)(run + ex);
      if (run + ex + sz <= (uint32_t)LZ_BLK) {  // beyond: the block goes out raw anyway
        const int lstart = (int)(e.x & 0xFFFFu), L = (int)(e.x >> 16);
        const int M = s + 1 < ns ? (int)(e.y >> 16) - 4 : 0;
        lz_put(ob, pos++, (uint32_t)((L >= 15 ? 15 : L) << 4) | (uint32_t)(M >= 15 ? 15 : M));
        if (L >= 15) {
          int r = L - 15;
          for (; r >= 255; r -= 255) lz_put(ob, pos++, 255u);
          lz_put(ob, pos++, (uint32_t)r);
        }
        for (int t = 0; t < L; ++t) lz_put(ob, pos++, lz_byte(S.data, lstart + t));
        if (s + 1 < ns) {
          const uint32_t off = e.y & 0xFFFFu;
          lz_put(ob, pos++, off & 0xFFu);
          lz_put(ob, pos++, off >> 8);
          if (M >= 15) {
            int r = M - 15;
            for (; r >= 255; r -= 255) lz_put(ob, pos++, 255u);
            lz_put(ob, pos++, (uint32_t)r);
          }
        }
      }
    }
    run += tot;
  }
  __syncthreads();
  const bool raw = run >= (uint32_t)len;
  uint8_t* dst = slots + blk * LZ_BLK_OUT;
  const int outn = raw ? len : (int)run;
  for (int t = lane; t < outn; t += 64) dst[t] = raw ? (uint8_t)lz_byte(S.data, hist + t) : ob[t];
  if (lane == 0) bsize[blk] = (uint32_t)outn | (raw ? 0x80000000u : 0u);
}

// frame assembly: block offsets (one block scans), header, size-prefixed blocks, end mark
__global__ void __launch_bounds__(256) lz4_frame_offsets(const uint32_t* __restrict__ bsize,
                                                         int64_t nblk, uint64_t* __restrict__ boff,
                                                         uint64_t* __restrict__ total) {
  __shared__ uint64_t wsum[4];
  uint64_t run = LZ_HDR;
  for (int64_t b0 = 0; b0 < nblk; b0 += 256) {
    const int64_t b = b0 + threadIdx.x;
    const uint64_t v = b < nblk ? 4ull + (bsize[b] & 0x7FFFFFFFu) : 0ull;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot);
    if (b < nblk) boff[b] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) *total = run + 4;  // + end mark
}

__global__ void __launch_bounds__(256) lz4_frame_write(const uint8_t* __restrict__ slots,
                                                       const uint32_t* __restrict__ bsize,
                                                       const uint64_t* __restrict__ boff,
                                                       const uint64_t* __restrict__ total,
                                                       int64_t nblk, uint8_t* __restrict__ out,
                                                       uint32_t hdr_lo, uint32_t hdr_mid,
                                                       uint64_t content) {
  const int64_t b = blockIdx.x;
  if (b == 0 && threadIdx.x < LZ_HDR) {
    const int t = threadIdx.x;
    uint8_t v;
    if (t < 4) v = (uint8_t)(LZ_MAGIC >> (8 * t));
    else if (t == 4) v = (uint8_t)(hdr_lo & 0xFF);          // FLG
    else if (t == 5) v = (uint8_t)((hdr_lo >> 8) & 0xFF);   // BD
    else if (t < 14) v = (uint8_t)(content >> (8 * (t - 6)));
    else v = (uint8_t)(hdr_mid & 0xFF);                     // HC
    out[t] = v;
  }
  if (b == 0 && threadIdx.x < 4) out[*total - 4 + threadIdx.x] = 0;  // end mark
  if (b >= nblk) return;
  const uint32_t sz = bsize[b];
  const uint64_t o = boff[b];
  if (threadIdx.x < 4) out[o + threadIdx.x] = (uint8_t)(sz >> (8 * threadIdx.x));
  const uint32_t m = sz & 0x7FFFFFFFu;
  const uint8_t* src = slots + b * LZ_BLK_OUT;
  for (uint32_t t = threadIdx.x; t < m; t += 256) out[o + 4 + t] = src[t];
}

// ---- decoder ----------------------------------------------------------------------------------
// One workgroup (64 threads) decodes the blocks [b0, b1) in order (b1 = b0 + 1 for independent
// frames) with an LDS ring of the last 64 KB decoded (an LZ4 offset is < 2^16, and a match copy
// never overwrites a ring slot it still has to read: the slot of position p is rewritten by
// p + 65536 only).  Output goes to a per-block slot (independent) or out + the running offset
// (linked).  The compressed block is staged in LDS.
struct LzBlock {
  int64_t in_off;   // first byte of the block data (after its 4-byte size)
  uint32_t csize;   // compressed size
  uint32_t raw;     // stored uncompressed
};

// the block just decoded, ring positions [a, b) (b - a <= ring size), to out[a .. b): bytes up to
// a 16-byte boundary of the output, then 16-byte stores of bytes gathered from the ring
__device__ __forceinline__ void lz4_ring_out(const uint8_t* ring, uint32_t wmask, uint64_t a,
                                             uint64_t b, uint8_t* out, uint64_t cap) {
  const int lane = threadIdx.x;
  if (b > cap) b = cap;
  if (a >= b) return;
  const uint64_t head = ((16 - ((uintptr_t)(out + a) & 15)) & 15);
  const uint64_t a16 = a + head < b ? a + head : b;
  for (uint64_t p = a + lane; p < a16; p += 64) out[p] = ring[p & wmask];
  const uint64_t nv = (b - a16) / 16;
  for (uint64_t v = lane; v < nv; v += 64) {
    const uint64_t p = a16 + 16 * v;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t pq = p + 4 * q;
      w[q] = (uint32_t)ring[pq & wmask] | ((uint32_t)ring[(pq + 1) & wmask] << 8) |
             ((uint32_t)ring[(pq + 2) & wmask] << 16) | ((uint32_t)ring[(pq + 3) & wmask] << 24);
    }
    *reinterpret_cast<uint4*>(out + p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (uint64_t p = a16 + 16 * nv + lane; p < b; p += 64) out[p] = ring[p & wmask];
}

// The token walk is wave-uniform scalar work: the next 256 bytes of the staged block sit one
// word per lane in a register window (refilled with one LDS read when the walk passes its end),
// and a byte is a v_readlane away — no LDS round trip per token / length / offset byte.  Literal
// and match bytes are copied by the whole wave inside the LDS ring (one wave per workgroup, so
// its LDS accesses stay in program order without barriers).
struct LzWin {
  uint32_t wv;     // this lane's word: staged bytes [base + 4 lane, +4)
  uint32_t base;   // window start (a multiple of 4)
};

__device__ __forceinline__ uint32_t lz_win_byte(LzWin& w, const uint32_t* cb32, uint32_t p) {
  if (p - w.base >= 252u) {  // (unsigned: also p < base, which never happens)
    w.base = p & ~3u;
    w.wv = cb32[(w.base >> 2) + threadIdx.x];
  }
  const uint32_t r = p - w.base;
  return (__builtin_amdgcn_readlane(w.wv, (int)(r >> 2)) >> (8 * (r & 3))) & 0xFFu;
}

// flagged_only (independent frames): decode only the blocks lz4_decode_par_kernel left to it
// (dsize[b] == LZ_PAR_FALLBACK); the other workgroups leave at once.
constexpr uint64_t LZ_PAR_FALLBACK = ~0ull;

__global__ void __launch_bounds__(64) lz4_decode_kernel(const uint8_t* __restrict__ in,
                                                        const LzBlock* __restrict__ blocks,
                                                        int64_t nblk, int linked, uint32_t bmax,
                                                        uint32_t win, uint8_t* __restrict__ out,
                                                        uint64_t out_cap,
                                                        uint64_t* __restrict__ dsize,
                                                        uint32_t* __restrict__ status,
                                                        int flagged_only) {
  if (flagged_only && !linked && dsize[blockIdx.x] != LZ_PAR_FALLBACK) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lz_smem[];
  uint8_t* ring = lz_smem;           // win bytes
  uint8_t* cb = lz_smem + win;       // staged compressed block (+ 256 bytes of window slack)
  const uint32_t* cb32 = reinterpret_cast<const uint32_t*>(cb);
  const int lane = threadIdx.x;
  const uint32_t wmask = win - 1;
  int64_t b0 = linked ? 0 : blockIdx.x, b1 = linked ? nblk : blockIdx.x + 1;
  uint64_t opos = 0;                 // bytes decoded so far by this workgroup (ring position)
  uint64_t obase = linked ? 0 : (uint64_t)blockIdx.x * bmax;  // output slot
  bool bad = false;
  for (int64_t b = b0; b < b1 && !bad; ++b) {
    const LzBlock B = blocks[b];
    if (B.csize > bmax + 16 || (B.raw && B.csize > bmax)) { bad = true; break; }
    lz_stage(cb, in + B.in_off, B.csize);
    for (uint32_t t = B.csize + lane; t < B.csize + 256; t += 64) cb[t] = 0;
    __syncthreads();
    const uint64_t start = opos;
    if (B.raw) {
      for (uint32_t t = lane; t < B.csize; t += 64) ring[(opos + t) & wmask] = cb[t];
      opos += B.csize;
      __syncthreads();
      lz4_ring_out(ring, wmask, start, opos, out + obase, out_cap > obase ? out_cap - obase : 0);
      if (!linked && lane == 0) dsize[b] = opos - start;
      continue;
    }
    LzWin w{cb32[lane], 0u};
    uint32_t ip = 0;
    const uint32_t cs = B.csize;
    for (;;) {  // wave-uniform token walk
      if (ip >= cs) { bad = true; break; }
      const uint32_t tok = lz_win_byte(w, cb32, ip++);
      uint32_t L = tok >> 4;
      if (L == 15) {
        uint32_t x;
        do {
          if (ip >= cs) { bad = true; break; }
          x = lz_win_byte(w, cb32, ip++);
          L += x;
        } while (x == 255);
        if (bad) break;
      }
      if (ip + L > cs || opos - start + L > bmax) { bad = true; break; }
      for (uint32_t t = lane; t < L; t += 64) ring[(opos + t) & wmask] = cb[ip + t];
      ip += L;
      opos += L;
      if (ip == cs) break;  // the last sequence has no match
      if (ip + 2 > cs) { bad = true; break; }
      const uint32_t off = lz_win_byte(w, cb32, ip) | (lz_win_byte(w, cb32, ip + 1) << 8);
      ip += 2;
      uint32_t M = (tok & 15u);
      if (M == 15) {
        uint32_t x;
        do {
          if (ip >= cs) { bad = true; break; }
          x = lz_win_byte(w, cb32, ip++);
          M += x;
        } while (x == 255);
        if (bad) break;
      }
      M += 4;
      const uint64_t hist = linked ? opos : opos - start;  // reachable history
      if (off == 0 || off > hist || opos - start + M > bmax) { bad = true; break; }
      // out[opos + t] = out[opos - off + (t mod off)]: each byte independently
      if (off >= M) {
        for (uint32_t t = lane; t < M; t += 64)
          ring[(opos + t) & wmask] = ring[(opos - off + t) & wmask];
      } else {
        for (uint32_t t = lane; t < M; t += 64)
          ring[(opos + t) & wmask] = ring[(opos - off + (t % off)) & wmask];
      }
      opos += M;
    }
    __syncthreads();
    if (!bad) lz4_ring_out(ring, wmask, start, opos, out + obase, out_cap > obase ? out_cap - obase : 0);
    if (!linked && lane == 0) dsize[b] = opos - start;
  }
  if (bad && lane == 0) atomicOr(status, 1u);
  if (linked && lane == 0) dsize[0] = opos;
}

// ---- parallel decode of a small independent block (this codec's frames: 2 KB blocks) --------
// The sequential decoder walks ≈ 500 sequences per 2 KB block of index gaps one after another,
// each costing a few dependent LDS / readlane steps (≈ 115 us per frame measured).  Here a
// 256-thread workgroup decodes the block with no sequential walk longer than a 64-byte chunk:
//  1. every byte position p is parsed AS IF a token started there: nxt[p] = the position after
//     its sequence (literal length and its extension bytes, literals, offset, match extension);
//  2. from every p, a walk along nxt until it leaves p's 64-byte chunk: exit[p];
//  3. one thread chains the chunks: 0 -> exit[0] -> exit[exit[0]] ... (one step per chunk),
//     which gives every chunk's true entry token;
//  4. each chunk re-walks from its entry and flags its true tokens;
//  5. a block scan of the tokens' decoded lengths gives each sequence's output offset;
//  6. every output byte gets its source: src = a compressed position (literal) or an earlier
//     output position (match byte at distance off); pointer jumping (src[p] = src[src[p]], in
//     place, <= log2(LZ_PAR_MAX) + 1 rounds) leaves every byte on a literal;
//  7. the bytes are read from the staged block and stored 4 at a time.
// A block that decodes past LZ_PAR_MAX bytes (or is stored raw, or larger) is left to the
// sequential kernel (dsize[b] = LZ_PAR_FALLBACK).  Every index is bounds-checked; a malformed
// block (a chain through an invalid parse, an offset before the block start) sets *status.
constexpr int LZ_PAR_MAX = 4096;                    // decoded bytes per block on this path
constexpr int LZ_PAR_CMAX = LZ_PAR_MAX + 64;        // compressed bytes per block on this path
constexpr int LZ_PAR_CHUNK = 64;                    // walk chunk (bytes of the compressed block)
constexpr int LZ_PAR_NCH = (LZ_PAR_CMAX + LZ_PAR_CHUNK - 1) / LZ_PAR_CHUNK;
constexpr int LZ_PAR_T = 1024;                      // threads per block: 4 waves per SIMD hide the
                                                    // LDS / VALU latency of each phase (1 block per CU)
constexpr int LZ_PAR_PPT = (LZ_PAR_CMAX + LZ_PAR_T - 1) / LZ_PAR_T;  // positions per thread
constexpr uint32_t LZ_LIT = 0x80000000u;            // src[p]: literal flag (| compressed pos)
constexpr uint32_t LZ_EXT = 0x40000000u;            // src[p]: an earlier block's byte (linked
                                                    // frames): | (65536 + source position
                                                    // relative to this block's start, < 0)
constexpr uint16_t LZ_BAD = 0xFFFFu;                // nxt[p]: no valid sequence at p
constexpr uint16_t LZ_BIG = 0xFFFEu;                // nxt[p]: decodes past LZ_PAR_MAX

struct LzParLds {
  uint32_t cb32[(LZ_PAR_CMAX + 256) / 4];  // staged compressed block + zero slack
  uint16_t nxt[LZ_PAR_CMAX];
  uint16_t ext[LZ_PAR_CMAX];
  uint16_t ooff[LZ_PAR_CMAX];              // output offset of the token at p (true tokens)
  uint8_t tok[LZ_PAR_CMAX];                // 1: a true token
  uint32_t src[LZ_PAR_MAX];
  uint16_t entry[LZ_PAR_NCH];
  uint32_t wsum[16];
  uint32_t total, state, changed;          // state: 0 ok, 1 bad, 2 fallback
};

#ifdef DPZ_STAMPS
__device__ unsigned long long g_lz_st[10][512];  // phase stamps of blocks < 512 (diagnostic build)
#define LZST(i) do { if (threadIdx.x == 0 && blockIdx.x < 512) g_lz_st[i][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define LZST(i) do {} while (0)
#endif

struct LzSeq {
  uint32_t lit, L, off, M, next;  // next = position after the sequence; kind in the caller
  int kind;                       // 0 sequence with a match, 1 last (literals only), 2 bad, 3 big
};

// The sequence a token at p would start (cb holds cs bytes + >= 256 zero bytes of slack).
__device__ __forceinline__ LzSeq lz_parse_at(const uint8_t* cb, uint32_t p, uint32_t cs) {
  LzSeq q{0, 0, 0, 0, 0, 2};
  const uint32_t tok = cb[p];
  uint32_t ip = p + 1, L = tok >> 4;
  if (L == 15) {
    uint32_t x;
    do {
      if (ip >= cs || L > (uint32_t)LZ_PAR_MAX) { q.kind = L > (uint32_t)LZ_PAR_MAX ? 3 : 2; return q; }
      x = cb[ip++];
      L += x;
    } while (x == 255);
  }
  if (L > (uint32_t)LZ_PAR_MAX) { q.kind = 3; return q; }
  if (ip + L > cs) return q;
  q.lit = ip;
  q.L = L;
  ip += L;
  if (ip == cs) {
    q.kind = 1;
    q.next = cs;
    return q;
  }
  if (ip + 2 > cs) return q;
  q.off = cb[ip] | ((uint32_t)cb[ip + 1] << 8);
  ip += 2;
  uint32_t M = tok & 15u;
  if (M == 15) {
    uint32_t x;
    do {
      if (ip >= cs || M > (uint32_t)LZ_PAR_MAX) { q.kind = M > (uint32_t)LZ_PAR_MAX ? 3 : 2; return q; }
      x = cb[ip++];
      M += x;
    } while (x == 255);
  }
  M += 4;
  if (M > (uint32_t)LZ_PAR_MAX) { q.kind = 3; return q; }
  if (ip > cs) return q;
  q.M = M;
  q.next = ip;
  q.kind = 0;
  return q;
}

// wslot (linked frames): per block LZ_PAR_MAX 32-bit words instead of the byte slots: a decoded
// byte, or LZ_EXT-style reference (bit 31 | (65536 + source position relative to the block
// start)) of a byte whose copy chain leaves the block (lz4_link_place / lz4_link_resolve finish it)
__global__ void __launch_bounds__(LZ_PAR_T) lz4_decode_par_kernel(const uint8_t* __restrict__ in,
                                                             const LzBlock* __restrict__ blocks,
                                                             uint32_t bmax,
                                                             uint8_t* __restrict__ slots,
                                                             uint64_t* __restrict__ dsize,
                                                             uint32_t* __restrict__ status,
                                                             uint32_t* __restrict__ wslot) {
  const bool linked = wslot != nullptr;
  __shared__ LzParLds S;
  const int t = threadIdx.x, wid = t >> 6;
  const int64_t b = blockIdx.x;
  const LzBlock B = blocks[b];
  uint8_t* cb = reinterpret_cast<uint8_t*>(S.cb32);
  if (linked && B.raw && B.csize <= (uint32_t)LZ_PAR_MAX) {  // a stored block: its bytes
    uint32_t* wd = wslot + (uint64_t)b * LZ_PAR_MAX;
    for (uint32_t p = t; p < B.csize; p += LZ_PAR_T) wd[p] = in[B.in_off + p];
    if (t == 0) dsize[b] = B.csize;
    return;
  }
  if (B.raw || B.csize > (uint32_t)LZ_PAR_CMAX || B.csize == 0) {  // the sequential kernel's
    if (t == 0) dsize[b] = LZ_PAR_FALLBACK;
    return;
  }
  const uint32_t cs = B.csize;
  LZST(0);
  {  // every wave stages a 1 KB slice (one round of loads in flight per lane)
    const uint32_t o = (uint32_t)wid * 1024u;
    if (o < cs) lz_stage(cb + o, in + B.in_off + o, cs - o < 1024u ? cs - o : 1024u);
  }
  for (uint32_t q = cs + t; q < cs + 256; q += LZ_PAR_T) cb[q] = 0;
  if (t == 0) {
    S.state = 0;
    S.total = 0;
  }
  __syncthreads();
  LZST(1);
  // 1. the sequence a token at every position would start: its length follows from the token
  // byte alone unless a length needs extension bytes (nibble 15); those positions (marked
  // LZ_SLOW) take the full parse in a second pass (no per-item arrays: nothing goes to scratch)
  constexpr uint16_t LZ_SLOW = 0xFFFDu;
  for (uint32_t p = t; p < cs; p += LZ_PAR_T) {
    const uint32_t tk = cb[p];
    const uint32_t L = tk >> 4, M = tk & 15u;
    uint16_t nx;
    if (L == 15 || M == 15) {
      nx = LZ_SLOW;
    } else {  // literals [p + 1, p + 1 + L), then the end of the block or a 2-byte offset
      const uint32_t ip = p + 1 + L;
      nx = ip > cs ? LZ_BAD : (ip == cs ? (uint16_t)cs : (ip + 2 > cs ? LZ_BAD : (uint16_t)(ip + 2)));
    }
    S.nxt[p] = nx;
    S.tok[p] = 0;
  }
  for (uint32_t p = t; p < cs; p += LZ_PAR_T) {
    if (S.nxt[p] != LZ_SLOW) continue;
    const LzSeq q = lz_parse_at(cb, p, cs);
    S.nxt[p] = q.kind <= 1 ? (uint16_t)q.next : (q.kind == 3 ? LZ_BIG : LZ_BAD);
  }
  for (int c = t; c < LZ_PAR_NCH; c += LZ_PAR_T) S.entry[c] = LZ_BAD;
  __syncthreads();
  LZST(2);
  // 2. from every position, the walk to the first position past its chunk (all of a thread's
  // walks advance in lockstep, branch-free, so their LDS reads are in flight together)
  {
    uint32_t cur[LZ_PAR_PPT];
#pragma unroll
    for (int i = 0; i < LZ_PAR_PPT; ++i) {
      const uint32_t p = t + (uint32_t)LZ_PAR_T * i;
      cur[i] = p < cs ? p : 0xFFFFFFFFu;
    }
    for (int step = 0; step < LZ_PAR_CHUNK; ++step) {
      bool any = false;
#pragma unroll
      for (int i = 0; i < LZ_PAR_PPT; ++i) {
        const uint32_t lim = ((t + (uint32_t)LZ_PAR_T * i) / LZ_PAR_CHUNK + 1) * LZ_PAR_CHUNK;
        const bool act = cur[i] < lim && cur[i] < cs;
        const uint32_t v = S.nxt[act ? cur[i] : 0u];  // > cur, or cs, or a marker
        cur[i] = act ? v : cur[i];
        any |= act;
      }
      if (!any) break;
    }
#pragma unroll
    for (int i = 0; i < LZ_PAR_PPT; ++i) {
      const uint32_t p = t + (uint32_t)LZ_PAR_T * i;
      if (p < cs) S.ext[p] = (uint16_t)(cur[i] > 0xFFFFu ? LZ_BAD : cur[i]);
    }
  }
  __syncthreads();
  LZST(3);
  // 3. the chain of chunk entries, one step per chunk
  if (t == 0) {
    uint32_t p = 0, st = 0, guard = 0;
    while (p < cs && guard++ < LZ_PAR_NCH + 1) {
      S.entry[p / LZ_PAR_CHUNK] = (uint16_t)p;
      const uint32_t x = S.ext[p];
      if (x == LZ_BAD) { st = 1; break; }
      if (x == LZ_BIG) { st = 2; break; }
      p = x;
    }
    if (!st && p != cs) st = 1;  // the last sequence must end the block exactly
    S.state = st;
  }
  __syncthreads();
  if (S.state) {
    if (t == 0) {
      if (S.state == 2) {
        dsize[b] = LZ_PAR_FALLBACK;
      } else {
        dsize[b] = 0;
        atomicOr(status, 1u);
      }
    }
    return;
  }
  LZST(4);
  // 4. each entered chunk flags its true tokens
  for (int c = t; c < LZ_PAR_NCH; c += LZ_PAR_T) {
    uint32_t p = S.entry[c];
    if (p == LZ_BAD) continue;
    const uint32_t lim = (uint32_t)(c + 1) * LZ_PAR_CHUNK;
    while (p < lim && p < cs) {
      S.tok[p] = 1;
      p = S.nxt[p];
    }
  }
  __syncthreads();
  LZST(5);
  // 5. output offsets: block scan of the true tokens' decoded lengths (positions in order;
  // thread t owns the contiguous positions [t * PPT, (t + 1) * PPT); the lengths are parked in
  // ooff, then overwritten by the offsets)
  {
    const uint32_t p0 = (uint32_t)t * LZ_PAR_PPT;
    uint32_t mine = 0;
    for (uint32_t p = p0; p < p0 + LZ_PAR_PPT && p < cs; ++p) {
      uint32_t len = 0;
      if (S.tok[p]) {
        const LzSeq q = lz_parse_at(cb, p, cs);
        len = q.L + q.M;
      }
      S.ooff[p] = (uint16_t)(len > 0xFFFFu ? 0xFFFFu : len);
      mine += len;
    }
    uint32_t tot;
    uint32_t run = block_excl_scan(mine, S.wsum, &tot);
    if (tot > (uint32_t)LZ_PAR_MAX) {
      if (t == 0) dsize[b] = LZ_PAR_FALLBACK;
      return;  // identical in every thread
    }
    for (uint32_t p = p0; p < p0 + LZ_PAR_PPT && p < cs; ++p) {
      const uint32_t len = S.ooff[p];
      S.ooff[p] = (uint16_t)run;
      run += len;
    }
    if (t == 0) S.total = tot;
  }
  __syncthreads();
  const uint32_t total = S.total;
  LZST(6);
  // 6. every output byte's source (offsets checked against the block's history)
  bool bad = false;
  for (uint32_t p = t; p < cs; p += LZ_PAR_T) {
    if (!S.tok[p]) continue;
    const LzSeq q = lz_parse_at(cb, p, cs);
    const uint32_t o = S.ooff[p];
    for (uint32_t j = 0; j < q.L; ++j) S.src[o + j] = LZ_LIT | (q.lit + j);
    if (q.kind == 0) {
      if (q.off == 0 || (!linked && q.off > o + q.L)) {
        bad = true;
        continue;
      }
      for (uint32_t j = 0; j < q.M; ++j) {
        const int32_t ps = (int32_t)(o + q.L + j) - (int32_t)q.off;  // >= -65535
        S.src[o + q.L + j] = ps >= 0 ? (uint32_t)ps : (LZ_EXT | (uint32_t)(65536 + ps));
      }
    }
  }
  if (bad) S.state = 1;
  __syncthreads();
  if (S.state) {
    if (t == 0) {
      dsize[b] = 0;
      atomicOr(status, 1u);
    }
    return;
  }
  LZST(7);
  // pointer jumping: every byte ends on a literal
  for (int round = 0; round < 14; ++round) {
    if (t == 0) S.changed = 0;
    __syncthreads();
    bool ch = false;
    for (uint32_t p = t; p < total; p += LZ_PAR_T) {
      const uint32_t v = S.src[p];
      if (!(v & (LZ_LIT | LZ_EXT))) {
        const uint32_t u = S.src[v];  // v < p: an earlier output byte
        S.src[p] = u;
        ch |= !(u & (LZ_LIT | LZ_EXT));
      }
    }
    if (ch) S.changed = 1;
    __syncthreads();
    if (!S.changed) break;
    __syncthreads();
  }
  LZST(8);
  if (linked) {  // 7'. words out: a decoded byte, or (bit 31) a reference into earlier blocks
    uint32_t* wd = wslot + (uint64_t)b * LZ_PAR_MAX;
    for (uint32_t p = t; p < total; p += LZ_PAR_T) {
      const uint32_t v = S.src[p];
      wd[p] = (v & LZ_LIT) ? (uint32_t)cb[v & 0x7FFFu] : (0x80000000u | (v & 0x1FFFFu));
    }
    if (t == 0) dsize[b] = total;
    return;
  }
  // 7. bytes out: 4 per thread per step, one 32-bit store when whole
  uint8_t* dst = slots + (uint64_t)b * bmax;
  for (uint32_t p0 = 4 * t; p0 < total; p0 += 4 * LZ_PAR_T) {
    uint32_t wv = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t p = p0 + e;
      if (p < total) {
        const uint32_t v = S.src[p];
        const uint32_t c = (v & LZ_LIT) ? cb[v & 0x7FFFu] : 0u;
        wv |= c << (8 * e);
      }
    }
    if (p0 + 4 <= total) *reinterpret_cast<uint32_t*>(dst + p0) = wv;
    else
      for (uint32_t e = 0; p0 + e < total; ++e) dst[p0 + e] = (uint8_t)(wv >> (8 * e));
  }
  if (t == 0) dsize[b] = total;
  LZST(9);
}

#ifdef DPZ_STAMPS
extern "C" int dpz_debug_lz4_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_lz_st), sizeof(g_lz_st));
}
#endif

// ---- linked frames on the parallel path ------------------------------------------------------
// After lz4_decode_par_kernel (wslot), every block's words go to their frame position P (prefix of
// the decoded sizes): w[P] = the byte, or bit 31 | the frame position its copy chain reaches in an
// earlier block.  A block the parallel decoder left (FALLBACK) or an offset before the frame's
// start sets *status (bit 1: re-decode the frame sequentially; bit 0: malformed).
__global__ void __launch_bounds__(256) lz4_link_place_kernel(const uint32_t* __restrict__ wslot,
                                                             const uint64_t* __restrict__ dsize,
                                                             int64_t nblk, uint32_t* __restrict__ w,
                                                             uint64_t wcap, uint64_t* __restrict__ total,
                                                             uint32_t* __restrict__ status) {
  __shared__ uint64_t wsum[4];
  __shared__ uint64_t base_sh;
  __shared__ uint32_t fb_sh;
  const int64_t b = blockIdx.x;
  if (threadIdx.x == 0) fb_sh = 0;
  __syncthreads();
  uint64_t before = 0;
  for (int64_t c0 = 0; c0 < nblk; c0 += 256) {
    const int64_t c = c0 + threadIdx.x;
    const uint64_t d = c < nblk ? dsize[c] : 0ull;
    if (d == LZ_PAR_FALLBACK) fb_sh = 1;
    const uint64_t v = d == LZ_PAR_FALLBACK ? 0ull : d;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot);
    if (c == b) base_sh = before + ex;
    before += tot;
  }
  __syncthreads();
  if (fb_sh) {
    if (b == 0 && threadIdx.x == 0) atomicOr(status, 2u);
    return;
  }
  const uint64_t o = base_sh, m = dsize[b];
  bool bad = false;
  const uint32_t* wd = wslot + (uint64_t)b * LZ_PAR_MAX;
  for (uint64_t t = threadIdx.x; t < m; t += 256) {
    if (o + t >= wcap) {
      bad = true;
      break;
    }
    uint32_t v = wd[t];
    if (v & 0x80000000u) {
      const int64_t rel = (int64_t)(v & 0x1FFFFu) - 65536;  // < 0: before the block's start
      const int64_t s = (int64_t)o + rel;
      if (s < 0) {
        bad = true;
        v = 0;
      } else {
        v = 0x80000000u | (uint32_t)s;
      }
    }
    w[o + t] = v;
  }
  if (bad) atomicOr(status, 1u);
  if (b == 0 && threadIdx.x == 0) *total = before;
}

// Every referencing word follows its chain to a byte: pointer jumping in place (each step reads the
// referenced word: a byte ends the chain, a reference is followed; the word is rewritten with how
// far it got, so later readers skip ahead).  References point strictly backwards and a byte never
// changes, so any interleaving of the steps is correct; ``steps`` bounds a pass (0: to the end).
// The last pass also writes the bytes out.
__global__ void __launch_bounds__(256) lz4_link_resolve_kernel(uint32_t* __restrict__ w,
                                                               const uint64_t* __restrict__ total,
                                                               const uint32_t* __restrict__ status,
                                                               int steps, uint8_t* __restrict__ out,
                                                               uint64_t out_cap) {
  if (*status) return;
  const uint64_t n = *total;
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < n;
       p += (uint64_t)gridDim.x * 256) {
    uint32_t v = w[p];
    if (v & 0x80000000u) {
      for (int s = 0; steps == 0 || s < steps; ++s) {
        const uint32_t u = __hip_atomic_load(&w[v & 0x7FFFFFFFu], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        v = u;
        if (!(v & 0x80000000u)) break;
      }
      __hip_atomic_store(&w[p], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (out && p < out_cap) out[p] = (uint8_t)v;
  }
}

// independent frames: slot b (dsize[b] bytes at b * bmax) -> out + prefix
__global__ void __launch_bounds__(256) lz4_gather_kernel(const uint8_t* __restrict__ slots,
                                                         const uint64_t* __restrict__ dsize,
                                                         int64_t nblk, uint32_t bmax,
                                                         uint8_t* __restrict__ out,
                                                         uint64_t out_cap,
                                                         uint64_t* __restrict__ total) {
  __shared__ uint64_t wsum[4];
  __shared__ uint64_t base_sh;
  // every block recomputes the prefix of the sizes before its slot range (nblk is small)
  const int64_t b = blockIdx.x;
  uint64_t before = 0, all = 0;
  for (int64_t c0 = 0; c0 < nblk; c0 += 256) {
    const int64_t c = c0 + threadIdx.x;
    const uint64_t v = c < nblk ? dsize[c] : 0ull;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot);
    if (c == b) base_sh = before + ex;
    before += tot;
  }
  all = before;
  __syncthreads();
  const uint64_t o = base_sh, m = dsize[b];
  for (uint64_t t = threadIdx.x; t < m; t += 256)
    if (o + t < out_cap) out[o + t] = slots[(uint64_t)b * bmax + t];
  if (b == 0 && threadIdx.x == 0) *total = all;
}


// ---- index deltas (Lz4Wrapper.compress: np.diff(sorted, prepend=0)) and their running sum ----
__global__ void __launch_bounds__(256) delta_i32_kernel(const int32_t* __restrict__ in, int64_t k,
                                                        int32_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256)
    out[j] = (int32_t)((uint32_t)in[j] - (j ? (uint32_t)in[j - 1] : 0u));  // int32 wrap as numpy
}

constexpr int PS_TILE = 4096;  // elements per block of the running-sum kernels

__global__ void __launch_bounds__(256) psum_tiles_kernel(const int32_t* __restrict__ in, int64_t k,
                                                         int64_t* __restrict__ tsum) {
  __shared__ uint64_t wsum[4];
  const int64_t t0 = (int64_t)blockIdx.x * PS_TILE;
  int64_t acc = 0;
  for (int e = threadIdx.x; e < PS_TILE; e += 256)
    if (t0 + e < k) acc += in[t0 + e];
  uint64_t tot;
  block_excl_scan64((uint64_t)acc, wsum, &tot);
  if (threadIdx.x == 0) tsum[blockIdx.x] = (int64_t)tot;
}

__global__ void __launch_bounds__(256) psum_scan_kernel(int64_t* __restrict__ tsum, int64_t nt) {
  __shared__ uint64_t wsum[4];
  uint64_t run = 0;
  for (int64_t b0 = 0; b0 < nt; b0 += 256) {
    const int64_t b = b0 + threadIdx.x;
    const uint64_t v = b < nt ? (uint64_t)tsum[b] : 0ull;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot);
    if (b < nt) tsum[b] = (int64_t)(run + ex);
    run += tot;
  }
}

// inclusive running sum: out64[j] = sum in[0..j] (int64, numpy's cumsum of int32), out32 too
__global__ void __launch_bounds__(256) psum_write_kernel(const int32_t* __restrict__ in, int64_t k,
                                                         const int64_t* __restrict__ tsum,
                                                         int64_t* out64, int32_t* out32) {
  __shared__ uint64_t wsum[4];
  const int64_t t0 = (int64_t)blockIdx.x * PS_TILE;
  constexpr int PER = PS_TILE / 256;
  int64_t v[PER];
  int64_t acc = 0;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int64_t j = t0 + (int64_t)threadIdx.x * PER + e;
    v[e] = j < k ? in[j] : 0;
    acc += v[e];
  }
  uint64_t tot;
  int64_t run = tsum[blockIdx.x] + (int64_t)block_excl_scan64((uint64_t)acc, wsum, &tot);
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int64_t j = t0 + (int64_t)threadIdx.x * PER + e;
    run += v[e];
    if (j < k) {
      if (out64) out64[j] = run;
      if (out32) out32[j] = (int32_t)run;
    }
  }
}

// xxHash32 (seed 0) of a short buffer: the frame descriptor checksum
static uint32_t xxh32_small(const uint8_t* p, int len) {
  const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                 P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  uint32_t h = P5 + (uint32_t)len;
  int i = 0;
  for (; i + 4 <= len; i += 4) {
    const uint32_t v = (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) |
                       ((uint32_t)p[i + 3] << 24);
    h += v * P3;
    h = rotl(h, 17) * P4;
  }
  for (; i < len; ++i) {
    h += p[i] * P5;
    h = rotl(h, 11) * P1;
  }
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_lz4_max_bytes(int64_t n) {
  if (n < 0) return -1;
  const int64_t nblk = (n + LZ_BLK - 1) / LZ_BLK;
  return LZ_HDR + nblk * (4 + LZ_BLK) + 4 + 16;
}

extern "C" size_t dpz_lz4_workspace_bytes(int64_t n, int64_t nblk_in, int64_t bmax) {
  // encoder: per-block slots + sizes + offsets; decoder: block table + sizes + slots
  const int64_t nb_e = (n + LZ_BLK - 1) / LZ_BLK + 1;
  const size_t enc = (size_t)nb_e * LZ_BLK_OUT + (size_t)nb_e * 4 + (size_t)nb_e * 8 + 64;
  // linked frames (bmax == 0): the parallel path's per-block words and frame-position words
  const size_t slot_b = bmax > 0 ? (size_t)bmax : 2 * (size_t)LZ_PAR_MAX * 4;
  const size_t dec = (size_t)(nblk_in + 1) * (sizeof(LzBlock) + 8) + (size_t)(nblk_in + 1) * slot_b + 512;
  const size_t w = enc > dec ? enc : dec;
  return (w + 255) & ~(size_t)255;
}

extern "C" int dpz_lz4_compress(const uint8_t* in, int64_t n, uint8_t* out, int64_t out_cap,
                                int64_t* nbytes_host, void* ws, size_t ws_bytes,
                                dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n < 0 || (n > 0 && !in) || !out || !nbytes_host) return DPZ_ERR_ARG;
  if (out_cap < dpz_lz4_max_bytes(n)) return DPZ_ERR_ARG;
  const int64_t nblk = (n + LZ_BLK - 1) / LZ_BLK;
  if (ws_bytes < dpz_lz4_workspace_bytes(n, 0, 0) || !ws) return DPZ_ERR_WORKSPACE;
  uint8_t* w8 = static_cast<uint8_t*>(ws);
  uint8_t* slots = w8;
  uint32_t* bsize = reinterpret_cast<uint32_t*>(w8 + (size_t)(nblk + 1) * LZ_BLK_OUT);
  uint64_t* boff = reinterpret_cast<uint64_t*>(
      w8 + (((size_t)(nblk + 1) * LZ_BLK_OUT + (size_t)(nblk + 1) * 4 + 7) & ~(size_t)7));
  uint64_t* total = boff + nblk + 1;
  // descriptor: FLG = version 01, C.Size, and B.Indep unless blocks reach into their history
  // (LZ_WIN > 0: linked blocks, python-lz4's default); BD = 64 KB max block
  uint8_t desc[10];
  desc[0] = 0x40 | (LZ_WIN > 0 ? 0 : 0x20) | 0x08;
  desc[1] = 0x40;
  for (int i = 0; i < 8; ++i) desc[2 + i] = (uint8_t)((uint64_t)n >> (8 * i));
  const uint32_t hc = (xxh32_small(desc, 10) >> 8) & 0xFF;
  if (nblk > 0) {
    DPZ_TIMED(DPZ_KT_LZ4, st, lz4_encode_blocks<<<(unsigned)nblk, 64, sizeof(LzEncLds), st>>>(
                                  in, n, slots, bsize));
  }
  DPZ_TIMED(DPZ_KT_LZ4, st, lz4_frame_offsets<<<1, 256, 0, st>>>(bsize, nblk, boff, total));
  DPZ_TIMED(DPZ_KT_LZ4, st, lz4_frame_write<<<(unsigned)(nblk > 0 ? nblk : 1), 256, 0, st>>>(
                                slots, bsize, boff, total, nblk, out,
                                (uint32_t)desc[0] | ((uint32_t)desc[1] << 8), hc, (uint64_t)n));
  uint64_t tot = 0;
  DPZ_HIP_TRY(hipMemcpyAsync(&tot, total, 8, hipMemcpyDeviceToHost, st));
  DPZ_HIP_TRY(hipStreamSynchronize(st));
  *nbytes_host = (int64_t)tot;
  return DPZ_OK;
}

extern "C" int dpz_lz4_frame_info(const uint8_t* frame_host, int64_t nbytes, int64_t* content_size,
                                  int64_t* nblk, int* linked, int64_t* block_max) {
  if (!frame_host || nbytes < 7 || !content_size || !nblk || !linked || !block_max)
    return DPZ_ERR_ARG;
  const uint8_t* p = frame_host;
  const uint32_t magic = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
  if (magic != LZ_MAGIC) return DPZ_ERR_ARG;
  const uint8_t flg = p[4], bd = p[5];
  if ((flg >> 6) != 1 || (flg & 0x02) || (bd & 0x8F)) return DPZ_ERR_ARG;
  const int bmax_id = (bd >> 4) & 7;
  if (bmax_id < 4) return DPZ_ERR_ARG;
  const bool csize = flg & 0x08, dict = flg & 0x01, bsum = flg & 0x10;
  int64_t pos = 6;
  int64_t cs = -1;
  if (csize) {
    if (nbytes < pos + 8) return DPZ_ERR_ARG;
    cs = 0;
    for (int i = 0; i < 8; ++i) cs |= (int64_t)p[pos + i] << (8 * i);
    pos += 8;
  }
  if (dict) pos += 4;
  if (nbytes < pos + 1) return DPZ_ERR_ARG;
  if ((uint8_t)((xxh32_small(p + 4, (int)(pos - 4)) >> 8) & 0xFF) != p[pos]) return DPZ_ERR_ARG;
  pos += 1;
  int64_t nb = 0;
  for (;;) {
    if (nbytes < pos + 4) return DPZ_ERR_ARG;
    const uint32_t sz = p[pos] | (p[pos + 1] << 8) | (p[pos + 2] << 16) | ((uint32_t)p[pos + 3] << 24);
    pos += 4;
    if (sz == 0) break;
    pos += (sz & 0x7FFFFFFFu) + (bsum ? 4 : 0);
    if (pos > nbytes) return DPZ_ERR_ARG;
    ++nb;
  }
  *content_size = cs;
  *nblk = nb;
  *linked = (flg & 0x20) ? 0 : 1;
  *block_max = (int64_t)1 << (8 + 2 * bmax_id);
  return DPZ_OK;
}

extern "C" int dpz_lz4_decompress(const uint8_t* frame_dev, const uint8_t* frame_host,
                                  int64_t nbytes, uint8_t* out, int64_t out_cap,
                                  int64_t* n_host, void* ws, size_t ws_bytes,
                                  dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!frame_dev || !n_host || out_cap < 0 || (out_cap > 0 && !out)) return DPZ_ERR_ARG;
  int64_t cs, nb, bmax;
  int linked;
  int rc = dpz_lz4_frame_info(frame_host, nbytes, &cs, &nb, &linked, &bmax);
  if (rc != DPZ_OK) return rc;
  if (ws_bytes < dpz_lz4_workspace_bytes(0, nb, linked ? 0 : bmax) || !ws) return DPZ_ERR_WORKSPACE;
  const uint8_t flg = frame_host[4];
  const bool bsum = flg & 0x10;
  // block table from the host bytes, built in pinned memory (the H2D is a true async DMA): a
  // per-thread buffer of at most PIN_CAP bytes (freed when the thread exits; reused only after
  // this call's final synchronize), or, for a larger table, a pinned buffer of this call alone
  struct PinTab {
    void* p = nullptr;
    size_t cap = 0;
    ~PinTab() {
      if (p) (void)hipHostFree(p);
    }
  };
  constexpr size_t PIN_CAP = 64 * 1024;  // 4K blocks: a 16 MB frame of 4 KB blocks
  thread_local PinTab tab_tls;
  PinTab tab_call;  // an oversize table's buffer, freed on return
  const size_t tab_need = sizeof(LzBlock) * (size_t)(nb + 1) + 16;
  PinTab& pt = tab_need <= PIN_CAP ? tab_tls : tab_call;
  if (pt.cap < tab_need) {
    if (pt.p) (void)hipHostFree(pt.p);
    pt.p = nullptr;
    pt.cap = 0;
    const size_t want = tab_need <= PIN_CAP ? PIN_CAP : tab_need;
    if (hipHostMalloc(&pt.p, want) != hipSuccess || !pt.p) {
      pt.p = nullptr;
      return DPZ_ERR_INTERNAL;
    }
    pt.cap = want;
  }
  LzBlock* tab_h = static_cast<LzBlock*>(pt.p);
  int64_t pos = 6 + ((flg & 0x08) ? 8 : 0) + ((flg & 0x01) ? 4 : 0) + 1;
  for (int64_t b = 0; b < nb; ++b) {
    const uint8_t* p = frame_host + pos;
    const uint32_t sz = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
    tab_h[b].in_off = pos + 4;
    tab_h[b].csize = sz & 0x7FFFFFFFu;
    tab_h[b].raw = sz >> 31;
    pos += 4 + (sz & 0x7FFFFFFFu) + (bsum ? 4 : 0);
  }
  uint8_t* w8 = static_cast<uint8_t*>(ws);
  LzBlock* tab = reinterpret_cast<LzBlock*>(w8);
  uint64_t* dsize = reinterpret_cast<uint64_t*>(w8 + sizeof(LzBlock) * (size_t)(nb + 1));
  uint32_t* status = reinterpret_cast<uint32_t*>(dsize + nb + 1);
  uint64_t* total = reinterpret_cast<uint64_t*>(status + 2);
  uint8_t* slots = reinterpret_cast<uint8_t*>(total + 1);
  slots = reinterpret_cast<uint8_t*>(((uintptr_t)slots + 255) & ~(uintptr_t)255);
  uint32_t maxc_all = 0;
  for (int64_t b = 0; b < nb; ++b) maxc_all = maxc_all > tab_h[b].csize ? maxc_all : tab_h[b].csize;
  const uint32_t* csz = &maxc_all;
  hipError_t e = hipMemcpyAsync(tab, tab_h, sizeof(LzBlock) * (size_t)(nb > 0 ? nb : 1),
                                hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemsetAsync(status, 0, 16, st);
  // the pinned table is reused by the next call: every return below waits for this one's DMA
  struct SyncAtExit {
    hipStream_t s;
    ~SyncAtExit() { (void)hipStreamSynchronize(s); }
  } tab_guard{st};
  if (e != hipSuccess) return (int)e;
  uint64_t tot = 0;
  uint32_t bad = 0;
  bool done = false;  // the parallel linked path read back status and total already
  if (nb > 0) {
    // ring of 64 KB (smaller when every block is: independent frames whose block max is
    // smaller) + the largest compressed block
    const uint32_t maxc = *csz;
    const uint32_t win = 65536;
    const size_t shm = (size_t)win + (size_t)maxc + 16 + 256;
    if (bmax > 65536 || shm > 160 * 1024) return DPZ_ERR_UNSUPPORTED;
    DPZ_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(lz4_decode_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    // DPZ_LZ4_PAR=0: every independent block on the sequential decoder (diagnostic build)
    const bool par = DPZ_KNOB_INT(LZ4_PAR, 1) != 0;
    // linked frames whose blocks fit the parallel decoder (this codec's frames: 2 KB blocks
    // reaching 14 KB back): the blocks decode in parallel, references into earlier blocks are
    // resolved by pointer jumping over the whole frame; otherwise (python-lz4's 64 KB blocks, or
    // a block the parallel decoder leaves) one workgroup decodes the frame block after block
    bool par_linked = linked && par;
    for (int64_t bb = 0; bb < nb && par_linked; ++bb)
      par_linked = tab_h[bb].raw ? tab_h[bb].csize <= (uint32_t)LZ_PAR_MAX
                                 : tab_h[bb].csize <= (uint32_t)LZ_PAR_CMAX;
    if (par_linked) {
      uint32_t* wslot = reinterpret_cast<uint32_t*>(slots);
      uint32_t* wfr = wslot + (size_t)nb * LZ_PAR_MAX;
      const uint64_t wcap = (uint64_t)nb * LZ_PAR_MAX;
      DPZ_TIMED(DPZ_KT_LZ4, st, lz4_decode_par_kernel<<<(unsigned)nb, LZ_PAR_T, 0, st>>>(
                                    frame_dev, tab, (uint32_t)bmax, slots, dsize, status, wslot));
      DPZ_TIMED(DPZ_KT_LZ4, st, lz4_link_place_kernel<<<(unsigned)nb, 256, 0, st>>>(
                                    wslot, dsize, nb, wfr, wcap, total, status));
      int64_t g = (int64_t)((wcap + 255) / 256);
      if (g > 2048) g = 2048;
      for (int pass = 0; pass < 2; ++pass)  // bounded passes (path compression), then the end
        DPZ_TIMED(DPZ_KT_LZ4, st, lz4_link_resolve_kernel<<<(unsigned)g, 256, 0, st>>>(
                                      wfr, total, status, 16, nullptr, 0));
      DPZ_TIMED(DPZ_KT_LZ4, st, lz4_link_resolve_kernel<<<(unsigned)g, 256, 0, st>>>(
                                    wfr, total, status, 0, out, (uint64_t)out_cap));
      uint64_t back2[2] = {0, 0};
      DPZ_HIP_TRY(hipMemcpyAsync(back2, status, 16, hipMemcpyDeviceToHost, st));
      DPZ_HIP_TRY(hipStreamSynchronize(st));
      if ((uint32_t)back2[0] & 2u) {  // a block the parallel decoder left: decode sequentially
        DPZ_HIP_TRY(hipMemsetAsync(status, 0, 16, st));
        par_linked = false;
      } else {  // final: no second copy and synchronize (each costs a host round trip)
        bad = (uint32_t)back2[0];
        tot = back2[1];
        done = true;
      }
    }
    if (linked && !par_linked) {
      DPZ_TIMED(DPZ_KT_LZ4, st, lz4_decode_kernel<<<1, 64, shm, st>>>(
                                    frame_dev, tab, nb, 1, (uint32_t)bmax, win, out,
                                    (uint64_t)out_cap, total, status, 0));
    } else if (!linked) {
      if (par)
        DPZ_TIMED(DPZ_KT_LZ4, st, lz4_decode_par_kernel<<<(unsigned)nb, LZ_PAR_T, 0, st>>>(
                                      frame_dev, tab, (uint32_t)bmax, slots, dsize, status,
                                      nullptr));
      // the blocks the parallel decoder left (raw, large; all of them without it)
      DPZ_TIMED(DPZ_KT_LZ4, st, lz4_decode_kernel<<<(unsigned)nb, 64, shm, st>>>(
                                    frame_dev, tab, nb, 0, (uint32_t)bmax, win, slots,
                                    (uint64_t)nb * bmax, dsize, status, par ? 1 : 0));
      DPZ_TIMED(DPZ_KT_LZ4, st, lz4_gather_kernel<<<(unsigned)nb, 256, 0, st>>>(
                                    slots, dsize, nb, (uint32_t)bmax, out, (uint64_t)out_cap,
                                    total));
    }
    if (!done) {
      // status (4 bytes, padding) and total (8 bytes) are adjacent: one copy back
      uint64_t back[2] = {0, 0};
      DPZ_HIP_TRY(hipMemcpyAsync(back, status, 16, hipMemcpyDeviceToHost, st));
      DPZ_HIP_TRY(hipStreamSynchronize(st));
      bad = (uint32_t)back[0];
      tot = back[1];
    }
  }
  if (bad) return DPZ_ERR_ARG;
  if (cs >= 0 && (int64_t)tot != cs) return DPZ_ERR_ARG;
  if ((int64_t)tot > out_cap) return DPZ_ERR_WORKSPACE;
  *n_host = (int64_t)tot;
  return DPZ_OK;
}

extern "C" int dpz_delta_i32(const int32_t* in, int64_t k, int32_t* out, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (k < 0 || (k > 0 && (!in || !out)) || in == out) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  int64_t g = (k + 255) / 256;
  if (g > 4096) g = 4096;
  DPZ_TIMED(DPZ_KT_LZ4, st, delta_i32_kernel<<<(unsigned)g, 256, 0, st>>>(in, k, out));
  return DPZ_OK;
}

extern "C" size_t dpz_running_sum_workspace_bytes(int64_t k) {
  return (size_t)(((k + PS_TILE - 1) / PS_TILE) + 1) * 8 + 256;
}

extern "C" int dpz_running_sum_i32(const int32_t* in, int64_t k, int64_t* out64, int32_t* out32,
                                   void* ws, size_t ws_bytes, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (k < 0 || (k > 0 && (!in || (!out64 && !out32)))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  if (!ws || ws_bytes < dpz_running_sum_workspace_bytes(k)) return DPZ_ERR_WORKSPACE;
  const int64_t nt = (k + PS_TILE - 1) / PS_TILE;
  int64_t* tsum = static_cast<int64_t*>(ws);
  DPZ_TIMED(DPZ_KT_LZ4, st, psum_tiles_kernel<<<(unsigned)nt, 256, 0, st>>>(in, k, tsum));
  DPZ_TIMED(DPZ_KT_LZ4, st, psum_scan_kernel<<<1, 256, 0, st>>>(tsum, nt));
  DPZ_TIMED(DPZ_KT_LZ4, st, psum_write_kernel<<<(unsigned)nt, 256, 0, st>>>(in, k, tsum, out64, out32));
  return DPZ_OK;
}
