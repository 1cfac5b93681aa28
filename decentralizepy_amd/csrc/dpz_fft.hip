// Frequency-domain codec of the FFT sharing plugin: the real FFTs (hand-written mixed-radix
// Stockham passes, below) and the complex-coefficient kernels around the shared top-k / fold
// kernels.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/JWINS/FFT.py:12-25     change_transformer_fft: torch.fft.rfft(x)
//   sharing/JWINS/FFT.py:301       fft.irfft(total)  (normalisation "backward": 1/n on the inverse)
//   sharing/JWINS/FFT.py:143-156   topk(|change|) over complex64 coefficients, flat_fft[index]
//   sharing/PartialModel.py:315-329  acc += change / change += acc on the complex change
//   models/Model.py:53-64          accumulated_changes[indices] = 0 (complex)
//   sharing/JWINS/FFT.py:282-299   topkf = flat_fft.clone(); topkf[indices] = params  (fold input:
//                                  complex entries become float pairs for dpz_decode_average)
//
// Real FFT of n reals (round 6, native).  Even n: the n reals ARE M = n / 2 complex values
// z[j] = x[2j] + i x[2j+1]; Z = DFT_M(z), then one pass turns Z into the n / 2 + 1 coefficients
// X[k] = ((Z[k] + conj Z[M-k]) - i W_n^k (Z[k] - conj Z[M-k])) / 2 (pairs k, M - k in place); the
// inverse runs the same steps backwards (Im X[0], Im X[M] ignored, as pocketfft's c2r does) with
// 1/n folded into the last pass.  Odd n: a complex DFT of length n over (x, 0) / the Hermitian
// extension.  DFT_L is a Stockham autosort over GLOBAL passes of radix R <= 256 (the prime factors
// packed into as few passes as fit; a prime in 257..4096 gets a pass of its own): a block owns B
// consecutive columns j of a pass (B * R <= 4096 complex, B <= 16: 128-byte rows), loads the
// column elements in[j + r L / R] (row r: B consecutive complex), applies the pass twiddle
// W_{pR}^{r (j mod p)}, runs the column DFTs of length R in LDS as sub-passes of radix 2 / 4 / 8 /
// 3 / 5 / 7 / 11 / 13 (register butterflies; any other prime one output per thread), and stores
// out[(j / p) p R + (j mod p) + m p] (consecutive j: consecutive addresses).  Twiddles come from a
// two-level table W_nt^e = hi[e >> 11] * lo[e & 2047] (fp64-computed, rounded to fp32; cached per
// size like a plan).  Sizes with a prime factor above 4096 go to hipFFT (rocFFT) instead.
#include <hipfft/hipfft.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "dpz_common.h"
#include "dpz_knobs.h"
#include "dpz_topk.h"

namespace dpz {

// key[i] = |c[i]| after the accumulation step of DPZ_ACC_* (fp32, sqrt(re*re + im*im): the
// vectorised ATen-CPU complex abs; the FFT itself differs from pocketfft by rounding, so parity
// of this path is a tolerance parity).
template <int MODE>
__global__ void __launch_bounds__(256) cplx_key_kernel(const float2* __restrict__ change,
                                                       float2* acc, int64_t m,
                                                       float* __restrict__ key) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256) {
    float2 c = change[i];
    if (MODE == DPZ_ACC_ACCUMULATE) {
      float2 a = acc[i];
      a.x = a.x + c.x;
      a.y = a.y + c.y;
      acc[i] = a;
      c = a;
    } else if (MODE == DPZ_ACC_ADD) {
      const float2 a = acc[i];
      c.x = c.x + a.x;
      c.y = c.y + a.y;
    }
    const float re2 = c.x * c.x;
    const float im2 = c.y * c.y;
    key[i] = sqrtf(re2 + im2);  // correctly rounded (llvm.sqrt without afn)
  }
}

// out[j] = src[idx[j]]; acc[idx[j]] = 0 when acc is given (Model.rewind_accumulation)
__global__ void __launch_bounds__(256) cplx_gather_kernel(const float2* __restrict__ src, int64_t m,
                                                          const int32_t* __restrict__ idx,
                                                          int64_t k, float2* __restrict__ out,
                                                          float2* acc) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t i = idx[j];
    float2 v = make_float2(0.f, 0.f);
    if (i >= 0 && i < m) {
      v = src[i];
      if (acc) acc[i] = make_float2(0.f, 0.f);
    }
    out[j] = v;
  }
}

// pair[2j] = 2 idx[j], pair[2j + 1] = 2 idx[j] + 1: complex entries as float-pair entries
__global__ void __launch_bounds__(256) cplx_pair_idx_kernel(const int32_t* __restrict__ idx,
                                                            int64_t k, int32_t* __restrict__ pair) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int32_t i = idx[j];
    reinterpret_cast<int2*>(pair)[j] = make_int2(2 * i, 2 * i + 1);
  }
}

__global__ void __launch_bounds__(256) scale_kernel(float* x, int64_t n, float s) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    x[i] = x[i] * s;
}

static unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---- native mixed-radix FFT -------------------------------------------------------------------
constexpr int FT_THREADS = 256;
constexpr int FT_ELEMS = 2048;  // B * R complex per block (two LDS buffers of B * (R + 1))
constexpr int FT_REG_ELEMS = 2048;  // tiles up to this size load / store through registers
#ifndef DPZ_FT_IP_WAVES
#define DPZ_FT_IP_WAVES 5
#endif
constexpr int FT_MAXR = 4096;   // the largest prime a pass takes (larger: hipFFT)
constexpr int FT_PACK = 256;    // the largest packed radix of a pass
constexpr int FT_MAXPASS = 12;
constexpr int FT_MAXSUB = 12;
constexpr int FT_LO = 2048;     // two-level twiddle table: W^e = hi[e >> 11] * lo[e & 2047]

// roots of unity W_nt^e = exp(-2 pi i e / nt), e < nt (conjugated for the inverse)
struct FtTw {
  const float2* lo;
  const float2* hi;
  uint32_t nt;
};

__device__ __forceinline__ float2 ft_cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}

__device__ __forceinline__ float2 ft_root(const FtTw& t, uint32_t e, bool inv) {
  const float2 h = t.hi[e >> 11], l = t.lo[e & (FT_LO - 1)];
  float2 w = ft_cmul(h, l);
  if (inv) w.y = -w.y;
  return w;
}

struct FtPass {
  const float2* in;     // complex input (load modes 0 / 2)
  const float* in_re;   // real input (load mode 1)
  float2* out;          // complex output (store modes 0 / 1 / 3)
  float* out_re;        // real output (store mode 2)
  int64_t L;            // transform length
  int64_t S;            // L / R: columns (and the input row stride)
  int64_t p;            // product of the earlier passes' radices
  int R, B, RP;         // radix, columns per block (a power of two <= 16), LDS column pitch
  int nsub;
  int q[FT_MAXSUB];     // the LDS sub-passes' radices (product R)
  uint32_t mnb[FT_MAXSUB], mpp[FT_MAXSUB];  // u / (R / q) and u / pp as umulhi(u, m) (u < 2^16)
  int load_mode;        // 0 complex, 1 real (x, 0), 2 Hermitian extension of n_aux / 2 + 1 values,
                        // 3 the c2r pairing of X[0..n_aux] (even-n inverse, ft_c2r_pair)
  int store_mode;       // 0 complex, 1 complex * scale, 2 real part * scale, 3 indices < n_aux only
  int64_t n_aux;
  float scale;
  int inv;
  int pair;             // last pass of an even-n rfft: the block holds columns j and S - j and its
                        // stores are the X[k] / X[M - k] pairing (n_aux = M)
  FtTw tw;
};

__device__ __forceinline__ float2 ft_mi(float2 z, bool inv);
__device__ __forceinline__ float2 ft_c2r_pair(float2 p, float2 q, uint32_t kk, const FtTw& tw);
__device__ __forceinline__ float2 ft_r2c_pair(float2 p, float2 q, uint32_t kk, const FtTw& tw);

__device__ __forceinline__ float2 ft_load(const FtPass& a, int64_t i) {
  if (a.load_mode == 1) return make_float2(a.in_re[i], 0.0f);
  if (a.load_mode == 3) {  // Z[i] from X[i] and X[M - i] (Im X[0], Im X[M] dropped), as the
    float2 p = a.in[i], q = a.in[a.n_aux - i];  // separate pre pass computes it
    if (i == 0) {
      p.y = 0.0f;
      q.y = 0.0f;
    }
    return ft_c2r_pair(p, q, (uint32_t)i, a.tw);
  }
  if (a.load_mode == 2) {
    const int64_t h = a.n_aux / 2 + 1;
    if (i < h) {
      const float2 v = a.in[i];
      return i == 0 ? make_float2(v.x, 0.0f) : v;
    }
    const float2 v = a.in[a.n_aux - i];
    return make_float2(v.x, -v.y);
  }
  return a.in[i];
}

__device__ __forceinline__ void ft_store(const FtPass& a, int64_t o, float2 v) {
  switch (a.store_mode) {
    case 1: a.out[o] = make_float2(v.x * a.scale, v.y * a.scale); break;
    case 2: a.out_re[o] = v.x * a.scale; break;
    case 3: if (o < a.n_aux) a.out[o] = v; break;
    default: a.out[o] = v;
  }
}

// -i z (forward) / +i z (inverse)
__device__ __forceinline__ float2 ft_mi(float2 z, bool inv) {
  return inv ? make_float2(-z.y, z.x) : make_float2(z.y, -z.x);
}

// even-n forward pairing: X[k] = ((Z[k] + conj Z[M-k]) - i W_n^k (Z[k] - conj Z[M-k])) / 2 for
// p = Z[k], q = Z[M - k]
__device__ __forceinline__ float2 ft_r2c_pair(float2 p, float2 q, uint32_t kk, const FtTw& tw) {
  const float2 e = make_float2(p.x + q.x, p.y - q.y);
  const float2 d = make_float2(p.x - q.x, p.y + q.y);
  const float2 o = ft_mi(ft_cmul(ft_root(tw, kk, false), d), false);
  return make_float2(0.5f * (e.x + o.x), 0.5f * (e.y + o.y));
}

// even-n inverse pairing: Z[k] = (X[k] + conj X[M-k]) + i W_n^{-k} (X[k] - conj X[M-k]) for
// p = X[k], q = X[M - k]
__device__ __forceinline__ float2 ft_c2r_pair(float2 p, float2 q, uint32_t kk, const FtTw& tw) {
  const float2 e = make_float2(p.x + q.x, p.y - q.y);
  const float2 d = make_float2(p.x - q.x, p.y + q.y);
  const float2 o = ft_mi(ft_cmul(ft_root(tw, kk, true), d), true);
  return make_float2(e.x + o.x, e.y + o.y);
}

__device__ __forceinline__ void ft_dft4(float2& v0, float2& v1, float2& v2, float2& v3, bool inv) {
  const float2 a = make_float2(v0.x + v2.x, v0.y + v2.y), b = make_float2(v0.x - v2.x, v0.y - v2.y);
  const float2 c = make_float2(v1.x + v3.x, v1.y + v3.y);
  const float2 d = ft_mi(make_float2(v1.x - v3.x, v1.y - v3.y), inv);
  v0 = make_float2(a.x + c.x, a.y + c.y);
  v2 = make_float2(a.x - c.x, a.y - c.y);
  v1 = make_float2(b.x + d.x, b.y + d.y);
  v3 = make_float2(b.x - d.x, b.y - d.y);
}

template <int Q>
__device__ __forceinline__ void ft_dft(float2 (&v)[Q], const float2 (&w)[Q], bool inv) {
  if constexpr (Q == 2) {
    const float2 a = v[0], b = v[1];
    v[0] = make_float2(a.x + b.x, a.y + b.y);
    v[1] = make_float2(a.x - b.x, a.y - b.y);
  } else if constexpr (Q == 4) {
    ft_dft4(v[0], v[1], v[2], v[3], inv);
  } else if constexpr (Q == 8) {
    // two radix-4 DFTs (even / odd inputs), then y[m] = E[m] + W_8^m O[m], y[m+4] = E[m] - ...
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6], o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    ft_dft4(e0, e1, e2, e3, inv);
    ft_dft4(o0, o1, o2, o3, inv);
    constexpr float h = 0.70710678118654752f;
    const float2 t1 = inv ? make_float2(h * (o1.x - o1.y), h * (o1.x + o1.y))
                          : make_float2(h * (o1.x + o1.y), h * (o1.y - o1.x));
    const float2 t2 = ft_mi(o2, inv);
    const float2 t3 = inv ? make_float2(-h * (o3.x + o3.y), h * (o3.x - o3.y))
                          : make_float2(h * (o3.y - o3.x), -h * (o3.x + o3.y));
    v[0] = make_float2(e0.x + o0.x, e0.y + o0.y);
    v[4] = make_float2(e0.x - o0.x, e0.y - o0.y);
    v[1] = make_float2(e1.x + t1.x, e1.y + t1.y);
    v[5] = make_float2(e1.x - t1.x, e1.y - t1.y);
    v[2] = make_float2(e2.x + t2.x, e2.y + t2.y);
    v[6] = make_float2(e2.x - t2.x, e2.y - t2.y);
    v[3] = make_float2(e3.x + t3.x, e3.y + t3.y);
    v[7] = make_float2(e3.x - t3.x, e3.y - t3.y);
  } else {
    // odd prime: y[m] / y[Q-m] from a_r = v_r + v_{Q-r}, b_r = v_r - v_{Q-r} and W_Q^{mr} = (C, D):
    // v_r W^{mr} + v_{Q-r} W^{-mr} = C a_r + i D b_r
    constexpr int H = (Q - 1) / 2;
    float2 A[H + 1], Bv[H + 1];
    float2 y0 = v[0];
#pragma unroll
    for (int r = 1; r <= H; ++r) {
      A[r] = make_float2(v[r].x + v[Q - r].x, v[r].y + v[Q - r].y);
      Bv[r] = make_float2(v[r].x - v[Q - r].x, v[r].y - v[Q - r].y);
      y0 = make_float2(y0.x + A[r].x, y0.y + A[r].y);
    }
    float2 out[Q];
    out[0] = y0;
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      float cr = v[0].x, ci = v[0].y, dr = 0.0f, di = 0.0f;
#pragma unroll
      for (int r = 1; r <= H; ++r) {
        const float2 wr = w[(m * r) % Q];
        cr = fmaf(wr.x, A[r].x, cr);
        ci = fmaf(wr.x, A[r].y, ci);
        dr = fmaf(-wr.y, Bv[r].y, dr);
        di = fmaf(wr.y, Bv[r].x, di);
      }
      out[m] = make_float2(cr + dr, ci + di);
      out[Q - m] = make_float2(cr - dr, ci - di);
    }
    (void)inv;
#pragma unroll
    for (int m = 0; m < Q; ++m) v[m] = out[m];
  }
}

// x / d for x < 2^16, d <= 4096: umulhi(x, floor(2^32 / d) + 1) (exact in that range); m = 0
// stands for d = 1
__device__ __forceinline__ int ft_div(int x, uint32_t m) {
  return m ? (int)__umulhi((uint32_t)x, m) : x;
}

// W_R^e from the block's LDS table of the pass's R roots (R <= FT_PACK), else the global table
struct FtRoots {
  const float2* lds;  // W_R^e, e < R (nullptr: global)
  int R;
  uint32_t nt_over_r;
  __device__ __forceinline__ float2 get(const FtTw& tw, int e, bool inv) const {
    return lds ? lds[e] : ft_root(tw, (uint32_t)e * nt_over_r, inv);
  }
};

// one LDS sub-pass of radix Q over the block's B columns of length R: butterfly i of a column
// takes elements i + r R / Q, twiddles them by W_{pp Q}^{r (i mod pp)} = W_R^{r (i mod pp) R/(pp Q)},
// and writes the outputs to (i / pp) pp Q + (i mod pp) + m pp
template <int Q>
__device__ __forceinline__ void ft_sub(const float2* src, float2* dst, int B, int R, int RP, int pp,
                                       uint32_t mnb, uint32_t mpp, const FtRoots& rt,
                                       const FtTw& tw, bool inv) {
  const int nb = R / Q;
  const int sm = R / (pp * Q);
  float2 w[Q];
  if constexpr (Q != 2 && Q != 4 && Q != 8) {
#pragma unroll
    for (int m = 0; m < Q; ++m) w[m] = rt.get(tw, m * (R / Q), inv);
  }
  for (int u = threadIdx.x; u < B * nb; u += FT_THREADS) {
    const int c = ft_div(u, mnb), i = u - c * nb;
    const int ip = ft_div(i, mpp);
    const int k = i - ip * pp;
    const float2* s = src + c * RP + i;
    float2 v[Q];
#pragma unroll
    for (int r = 0; r < Q; ++r) v[r] = s[r * nb];
    if (k) {
#pragma unroll
      for (int r = 1; r < Q; ++r) v[r] = ft_cmul(v[r], rt.get(tw, r * k * sm, inv));
    }
    ft_dft<Q>(v, w, inv);
    float2* d = dst + c * RP + ip * pp * Q + k;
#pragma unroll
    for (int m = 0; m < Q; ++m) d[m * pp] = v[m];
  }
}

// the same sub-pass in place (one LDS buffer): each thread reads and transforms all its
// butterflies into registers, the block syncs, then the outputs are written over the inputs
template <int Q>
__device__ __forceinline__ void ft_sub_ip(float2* buf, int B, int R, int RP, int pp, uint32_t mnb,
                                          uint32_t mpp, const FtRoots& rt, const FtTw& tw,
                                          bool inv) {
  constexpr int NBT = (FT_REG_ELEMS / Q + FT_THREADS - 1) / FT_THREADS;
  const int nb = R / Q;
  const int sm = R / (pp * Q);
  float2 w[Q];
  if constexpr (Q != 2 && Q != 4 && Q != 8) {
#pragma unroll
    for (int m = 0; m < Q; ++m) w[m] = rt.get(tw, m * (R / Q), inv);
  }
  float2 v[NBT][Q];
  int dst[NBT];
#pragma unroll
  for (int b = 0; b < NBT; ++b) {
    const int u0 = threadIdx.x + b * FT_THREADS;
    const bool ok = u0 < B * nb;
    const int u = ok ? u0 : 0;
    const int c = ft_div(u, mnb), i = u - c * nb;
    const int ip = ft_div(i, mpp);
    const int k = i - ip * pp;
    const float2* s = buf + c * RP + i;
#pragma unroll
    for (int r = 0; r < Q; ++r) v[b][r] = s[r * nb];
    if (k) {
#pragma unroll
      for (int r = 1; r < Q; ++r) v[b][r] = ft_cmul(v[b][r], rt.get(tw, r * k * sm, inv));
    }
    ft_dft<Q>(v[b], w, inv);
    dst[b] = ok ? c * RP + ip * pp * Q + k : -1;
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < NBT; ++b) {
    if (dst[b] >= 0) {
#pragma unroll
      for (int m = 0; m < Q; ++m) buf[dst[b] + m * pp] = v[b][m];
    }
  }
}

// any other prime radix: one output per thread, O(q) terms
__device__ __forceinline__ void ft_sub_any(const float2* src, float2* dst, int B, int R, int RP,
                                           int pp, int q, const FtTw& tw, bool inv) {
  const int nb = R / q;
  const uint32_t sm = tw.nt / (uint32_t)(pp * q), sq = tw.nt / (uint32_t)q;
  for (int u = threadIdx.x; u < B * R; u += FT_THREADS) {
    const int c = u / R, rem = u - c * R;
    const int m = rem / nb, i = rem - m * nb;
    const int k = i % pp;
    const float2* s = src + c * RP + i;
    float accr = 0.0f, acci = 0.0f;
    for (int r = 0; r < q; ++r) {
      const uint64_t e = ((uint64_t)r * k * sm + (uint64_t)((r * m) % q) * sq) % tw.nt;
      const float2 z = ft_cmul(s[r * nb], ft_root(tw, (uint32_t)e, inv));
      accr += z.x;
      acci += z.y;
    }
    dst[c * RP + (i / pp) * pp * q + k + m * pp] = make_float2(accr, acci);
  }
}

// IP (in place): passes whose sub-radices are all in {2, 3, 4, 5, 7, 8} and whose tile goes
// through registers run with ONE LDS buffer (sub-passes staged in registers): 72 VGPRs and half
// the LDS, so more blocks per CU; the others (11, 13, other primes) ping-pong two buffers
extern __shared__ float2 ft_lds[];
template <bool IP>
__device__ __forceinline__ void ft_pass_body(const FtPass& a) {
  const int B = a.B, R = a.R, RP = a.RP;
  const int t = threadIdx.x;
  // pair mode: slots c < H hold columns jf0 + c (jf <= S / 2), slots H + c their mirrors S - jf
  // (column 0 is its own mirror: loaded twice)
  const int H = B >> 1;
  const int64_t j0 = a.pair ? (int64_t)blockIdx.x * H : (int64_t)blockIdx.x * B;
  const int cols = a.pair ? (int)(a.S / 2 - j0 + 1 < H ? a.S / 2 - j0 + 1 : H)
                          : (int)(a.S - j0 < B ? a.S - j0 : B);
  float2* src = ft_lds;
  float2* dst = IP ? ft_lds : ft_lds + B * RP;
  const bool inv = a.inv != 0;
  // the pass's R roots W_R^e in LDS (packed passes; a lone large prime reads the global table)
  FtRoots rt{nullptr, R, a.tw.nt / (uint32_t)R};
  if (R <= FT_PACK) {
    float2* tab = ft_lds + (IP ? 1 : 2) * B * RP;
    for (int e = t; e < R; e += FT_THREADS) tab[e] = ft_root(a.tw, (uint32_t)e * rt.nt_over_r, inv);
    rt.lds = tab;
  }
  // load: element (c, r) = in[j0 + c + r S], twiddled; B divides the block, so a thread's column
  // is the same for all its elements.  B * R <= FT_REG_ELEMS: every element's load (and its
  // twiddle's table loads) issued before the first is used, branch-free (an idle slot re-reads
  // column j0's first element); larger (a lone prime pass): element by element
  {
    const int c = t & (B - 1);
    int64_t j = j0 + c;
    bool cv = c < cols;
    if (a.pair) {
      const int cf = c < H ? c : c - H;
      const int64_t jf = j0 + cf;
      cv = cf < cols;
      j = (c < H || jf == 0) ? jf : a.S - jf;
    }
    const uint32_t k = a.p > 1 ? (uint32_t)(j % a.p) : 0u;
    const uint32_t twm = a.tw.nt / (uint32_t)(a.p * R);
    const int rs = FT_THREADS / B, r0 = t / B;
    if (B * R <= FT_REG_ELEMS) {
      float2 v[FT_REG_ELEMS / FT_THREADS], w[FT_REG_ELEMS / FT_THREADS];
#pragma unroll
      for (int i = 0; i < FT_REG_ELEMS / FT_THREADS; ++i) {
        const int r = r0 + i * rs;
        const bool ok = cv && r < R;
        v[i] = ft_load(a, ok ? j + (int64_t)r * a.S : j0);
        const uint32_t e = ok ? (uint32_t)(((uint64_t)r * k) * twm) : 0u;
        w[i] = ft_root(a.tw, e, inv);
      }
#pragma unroll
      for (int i = 0; i < FT_REG_ELEMS / FT_THREADS; ++i) {
        const int r = r0 + i * rs;
        if (cv && r < R) src[c * RP + r] = k ? ft_cmul(v[i], w[i]) : v[i];
      }
    } else if (cv) {
      for (int r = r0; r < R; r += rs) {
        float2 v = ft_load(a, j + (int64_t)r * a.S);
        if (k && r) v = ft_cmul(v, ft_root(a.tw, (uint32_t)(((uint64_t)r * k) * twm), inv));
        src[c * RP + r] = v;
      }
    }
  }
  __syncthreads();
  int pp = 1;
  for (int s = 0; s < a.nsub; ++s) {
    const int q = a.q[s];
    const uint32_t mn = a.mnb[s], mp = a.mpp[s];
    if constexpr (IP) {
      switch (q) {
        case 2: ft_sub_ip<2>(src, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 4: ft_sub_ip<4>(src, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 8: ft_sub_ip<8>(src, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 3: ft_sub_ip<3>(src, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 5: ft_sub_ip<5>(src, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        default: ft_sub_ip<7>(src, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
      }
      __syncthreads();
    } else {
      switch (q) {
        case 2: ft_sub<2>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 4: ft_sub<4>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 8: ft_sub<8>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 3: ft_sub<3>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 5: ft_sub<5>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 7: ft_sub<7>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 11: ft_sub<11>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        case 13: ft_sub<13>(src, dst, B, R, RP, pp, mn, mp, rt, a.tw, inv); break;
        default: ft_sub_any(src, dst, B, R, RP, pp, q, a.tw, inv);
      }
      __syncthreads();
      float2* x = src;
      src = dst;
      dst = x;
    }
    pp *= q;
  }
  // store: column j's output m to (j / p) p R + (j mod p) + m p; consecutive threads take
  // consecutive columns (p > 1) or consecutive outputs of one column (p = 1: a contiguous run);
  // the LDS reads of a thread's outputs all issued before its stores
  constexpr int NE = FT_REG_ELEMS / FT_THREADS;
  if (a.pair) {
    // output m of front column j is Z[o], o = j + m S; its partner Z[M - o] is output R - 1 - m
    // of the mirror column (column 0: output (R - m) mod R of itself); both X are written here
    const int64_t M = a.n_aux;
    const int cf = t & (H - 1);
    const int64_t j = j0 + cf;
    if (cf < cols) {
      for (int m = t / H; m < R; m += FT_THREADS / H) {
        const float2 zp = src[cf * RP + m];
        const int64_t o = j + (int64_t)m * a.S;
        if (o == 0) {
          a.out[0] = make_float2(zp.x + zp.y, 0.0f);
          a.out[M] = make_float2(zp.x - zp.y, 0.0f);
          continue;
        }
        const float2 zq = j == 0 ? src[cf * RP + (R - m)] : src[(cf + H) * RP + (R - 1 - m)];
        a.out[o] = ft_r2c_pair(zp, zq, (uint32_t)o, a.tw);
        a.out[M - o] = ft_r2c_pair(zq, zp, (uint32_t)(M - o), a.tw);
      }
    }
    return;
  }
  if (a.p == 1) {
    if (B * R <= FT_REG_ELEMS) {
      float2 v[NE];
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = t + i * FT_THREADS;
        const int c = e / R, m = e - c * R;
        v[i] = src[(c < B ? c : 0) * RP + m];
      }
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = t + i * FT_THREADS;
        const int c = e / R, m = e - c * R;
        if (c < cols) ft_store(a, (j0 + c) * R + m, v[i]);
      }
    } else {
      for (int e = t; e < cols * R; e += FT_THREADS) {
        const int c = e / R, m = e - c * R;
        ft_store(a, (j0 + c) * R + m, src[c * RP + m]);
      }
    }
  } else {
    const int c = t & (B - 1);
    const int64_t j = j0 + c;
    const int64_t base = (j / a.p) * a.p * R + j % a.p;
    const int rs = FT_THREADS / B, m0 = t / B;
    if (B * R <= FT_REG_ELEMS) {
      float2 v[NE];
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int m = m0 + i * rs;
        v[i] = src[c * RP + (m < R ? m : 0)];
      }
      if (c < cols) {
#pragma unroll
        for (int i = 0; i < NE; ++i) {
          const int m = m0 + i * rs;
          if (m < R) ft_store(a, base + (int64_t)m * a.p, v[i]);
        }
      }
    } else if (c < cols) {
      for (int m = m0; m < R; m += rs) ft_store(a, base + (int64_t)m * a.p, src[c * RP + m]);
    }
  }
}

// the in-place variant held to 5 waves per SIMD (96 VGPRs, 5 spilled; 6 waves spill 21 and run
// slower: rfft 181 vs 159 us at 11 M, profiles/r06_fft_inplace_ab.jsonl), the ping-pong one as it
// compiles (125 VGPRs, 4 waves)
__global__ void __launch_bounds__(FT_THREADS) __attribute__((amdgpu_waves_per_eu(DPZ_FT_IP_WAVES, 8)))
ft_pass_ip_kernel(FtPass a) {
  ft_pass_body<true>(a);
}
__global__ void __launch_bounds__(FT_THREADS) ft_pass_kernel(FtPass a) { ft_pass_body<false>(a); }

// even n, forward: X[k] = ((Z[k] + conj Z[M-k]) - i W_n^k (Z[k] - conj Z[M-k])) / 2 for the pair
// (k, M - k), k <= M / 2; Z read from `z` (may equal out)
__global__ void __launch_bounds__(256) ft_r2c_post_kernel(const float2* z, float2* out, int64_t M,
                                                          FtTw tw) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k <= M / 2; k += (int64_t)gridDim.x * 256) {
    if (k == 0) {
      const float2 z0 = z[0];
      out[0] = make_float2(z0.x + z0.y, 0.0f);
      out[M] = make_float2(z0.x - z0.y, 0.0f);
      continue;
    }
    const float2 a = z[k], b = z[M - k];
    const float2 xk = ft_r2c_pair(a, b, (uint32_t)k, tw);
    const float2 xm = ft_r2c_pair(b, a, (uint32_t)(M - k), tw);
    out[k] = xk;
    if (M - k != k) out[M - k] = xm;
  }
}

// even n, inverse: Z[k] = (X[k] + conj X[M-k]) + i W_n^{-k} (X[k] - conj X[M-k]) for the pair
// (k, M - k), Im X[0] = Im X[M] = 0 (c2r); `scale` multiplies (1 unless no pass follows)
__global__ void __launch_bounds__(256) ft_c2r_pre_kernel(const float2* x, float2* z, int64_t M,
                                                         FtTw tw, float scale) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k <= M / 2; k += (int64_t)gridDim.x * 256) {
    float2 a = x[k], b = x[M - k];
    if (k == 0) {
      a.y = 0.0f;
      b.y = 0.0f;
    }
    auto one = [&](float2 p, float2 q, int64_t kk) {  // p = X[kk], q = X[M - kk]
      const float2 z = ft_c2r_pair(p, q, (uint32_t)kk, tw);
      return make_float2(z.x * scale, z.y * scale);
    };
    const float2 zk = one(a, b, k);
    if (k == 0) {
      z[0] = zk;
      continue;
    }
    const float2 zm = one(b, a, M - k);
    z[k] = zk;
    if (M - k != k) z[M - k] = zm;
  }
}

struct FtPlan {
  int64_t L = 0;
  int npass = 0;
  int R[FT_MAXPASS];
  int nsub[FT_MAXPASS];
  int q[FT_MAXPASS][FT_MAXSUB];
};

// L = R_1 ... R_s: prime factors <= FT_PACK packed (largest first, each into the pass with the
// smallest product that stays <= FT_PACK), larger primes (<= FT_MAXR) a pass each; false when a
// prime exceeds FT_MAXR or the pass / sub-pass tables overflow
static bool ft_make_plan(int64_t L, FtPlan* pl) {
  pl->L = L;
  pl->npass = 0;
  if (L < 1) return false;
  std::vector<int64_t> primes;
  int64_t m = L;
  for (int64_t f = 2; f * f <= m; ++f)
    while (m % f == 0) {
      primes.push_back(f);
      m /= f;
    }
  if (m > 1) primes.push_back(m);
  // the packing bound (DPZ_FFT_PACK, diagnostic build: smaller passes of 128-byte rows, A/B)
  int64_t pack = DPZ_KNOB_INT(FFT_PACK, FT_PACK);
  if (pack < 2 || pack > FT_PACK) pack = FT_PACK;
  std::vector<std::vector<int>> bins;
  std::vector<int64_t> prod;
  std::sort(primes.begin(), primes.end(), std::greater<int64_t>());
  for (int64_t f : primes) {
    if (f > FT_MAXR) return false;
    if (f > pack) {
      bins.push_back({(int)f});
      prod.push_back(f);
      continue;
    }
    int best = -1;
    for (size_t b = 0; b < bins.size(); ++b)
      if (prod[b] <= pack && prod[b] * f <= pack && (best < 0 || prod[b] < prod[best])) best = (int)b;
    if (best < 0) {
      bins.push_back({(int)f});
      prod.push_back(f);
    } else {
      bins[best].push_back((int)f);
      prod[best] *= f;
    }
  }
  if ((int)bins.size() > FT_MAXPASS) return false;
  for (size_t b = 0; b < bins.size(); ++b) {
    // sub-passes: the 2s as radix 8 (then 4 / 2), the odd primes as themselves
    int twos = 0, ns = 0;
    int qs[FT_MAXSUB];
    for (int f : bins[b]) {
      if (f == 2) {
        ++twos;
      } else {
        if (ns == FT_MAXSUB) return false;
        qs[ns++] = f;
      }
    }
    while (twos > 0) {
      const int take = twos >= 3 ? 3 : twos;
      if (ns == FT_MAXSUB) return false;
      qs[ns++] = 1 << take;
      twos -= take;
    }
    pl->R[pl->npass] = (int)prod[b];
    pl->nsub[pl->npass] = ns;
    for (int i = 0; i < ns; ++i) pl->q[pl->npass][i] = qs[i];
    ++pl->npass;
  }
  return true;
}

// twiddle tables per (device, nt), like a plan: lo[e] = W_nt^e (e < 2048), hi[h] = W_nt^(2048 h)
struct FtTables {
  float2* lo = nullptr;
  float2* hi = nullptr;
};
static std::mutex g_ft_mu;
static std::map<std::pair<int, uint32_t>, FtTables> g_ft_tabs;

static int ft_tables(uint32_t nt, FtTw* tw) {
  int dev = 0;
  DPZ_HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(g_ft_mu);
  auto it = g_ft_tabs.find({dev, nt});
  if (it == g_ft_tabs.end()) {
    const size_t nhi = nt / FT_LO + 2;
    std::vector<float2> h(FT_LO + nhi);
    for (size_t e = 0; e < (size_t)FT_LO + nhi; ++e) {
      const uint64_t ex = e < (size_t)FT_LO ? e : (uint64_t)(e - FT_LO) * FT_LO;
      // angle 2 pi (ex mod nt) / nt in long double (exact reduction of the integer exponent)
      const long double th = 2.0L * 3.14159265358979323846264338327950288L *
                             (long double)(ex % nt) / (long double)nt;
      h[e] = make_float2((float)cosl(th), (float)-sinl(th));
    }
    FtTables t;
    float2* d = nullptr;
    DPZ_HIP_TRY(hipMalloc(&d, h.size() * sizeof(float2)));
    if (hipMemcpy(d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
      hipFree(d);
      return DPZ_ERR_INTERNAL;
    }
    t.lo = d;
    t.hi = d + FT_LO;
    it = g_ft_tabs.emplace(std::make_pair(dev, nt), t).first;
  }
  tw->lo = it->second.lo;
  tw->hi = it->second.hi;
  tw->nt = nt;
  return DPZ_OK;
}

static bool g_ft_lds_set = false;

// the plan's passes: pass 1 reads (in, in_re, load_mode), the last writes (out, out_re,
// store_mode, scale); the others alternate between bufA and bufB so that the last lands in out
static int ft_run(const FtPlan& pl, const FtTw& tw, bool inv, const float2* in, const float* in_re,
                  int load_mode, float2* out, float* out_re, int store_mode, float scale,
                  int64_t n_aux, float2* bufA, float2* bufB, hipStream_t st,
                  bool* pair_last = nullptr) {
  const bool want_pair = pair_last && *pair_last;
  if (pair_last) *pair_last = false;
  if (!g_ft_lds_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(ft_pass_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(ft_pass_ip_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return DPZ_ERR_INTERNAL;
    g_ft_lds_set = true;
  }
  int64_t p = 1;
  const float2* cur = in;
  for (int s = 0; s < pl.npass; ++s) {
    FtPass a{};
    const bool first = s == 0, last = s == pl.npass - 1;
    a.in = cur;
    a.in_re = in_re;
    a.load_mode = first ? load_mode : 0;
    a.L = pl.L;
    a.R = pl.R[s];
    a.S = pl.L / a.R;
    a.p = p;
    // columns per block: B * R <= FT_ELEMS (diagnostic knobs DPZ_FFT_ELEMS / DPZ_FFT_BMAX)
    const int elems = (int)DPZ_KNOB_INT(FFT_ELEMS, FT_ELEMS);
    int B = (int)DPZ_KNOB_INT(FFT_BMAX, 16);
    if (B < 1 || B > 16 || (B & (B - 1))) B = 16;
    while (B > 1 && (B * a.R > elems || B > 2 * a.S)) B >>= 1;
    a.B = B;
    a.RP = a.R + 1;
    a.nsub = pl.nsub[s];
    bool ip = B * a.R <= FT_REG_ELEMS && DPZ_KNOB_INT(FFT_INPLACE, 1) != 0;
    for (int i = 0; i < a.nsub; ++i) {
      const int q = pl.q[s][i];
      ip = ip && (q == 2 || q == 3 || q == 4 || q == 5 || q == 7 || q == 8);
    }
    int pp = 1;
    for (int i = 0; i < a.nsub; ++i) {
      a.q[i] = pl.q[s][i];
      const uint64_t nb = (uint64_t)(a.R / a.q[i]);
      a.mnb[i] = nb == 1 ? 0u : (uint32_t)((1ull << 32) / nb + 1);
      a.mpp[i] = pp == 1 ? 0u : (uint32_t)((1ull << 32) / (uint64_t)pp + 1);
      pp *= a.q[i];
    }
    a.n_aux = n_aux;
    a.scale = 1.0f;
    a.inv = inv ? 1 : 0;
    a.tw = tw;
    float2* dst;
    if (last) {
      dst = out;
      a.out_re = out_re;
      a.store_mode = store_mode;
      a.scale = scale;
    } else {
      dst = ((pl.npass - 1 - s) & 1) ? bufA : bufB;
      a.store_mode = 0;
    }
    a.out = dst;
    int64_t blocks = (a.S + B - 1) / B;
    if (last && want_pair && B >= 2) {  // the even-n rfft pairing in the last pass's stores
      a.pair = 1;
      a.n_aux = pl.L;
      blocks = (a.S / 2 + 1 + B / 2 - 1) / (B / 2);
      *pair_last = true;
    }
    const size_t lds = ((ip ? 1 : 2) * (size_t)B * a.RP + (a.R <= FT_PACK ? a.R : 0)) *
                       sizeof(float2);
    if (ip) {
      DPZ_TIMED(DPZ_KT_FFT, st, ft_pass_ip_kernel<<<(unsigned)blocks, FT_THREADS, lds, st>>>(a));
    } else {
      DPZ_TIMED(DPZ_KT_FFT, st, ft_pass_kernel<<<(unsigned)blocks, FT_THREADS, lds, st>>>(a));
    }
    cur = dst;
    p *= a.R;
  }
  return DPZ_OK;
}

// native plan of a real FFT of n reals: the complex length (M = n / 2 even, n odd) and whether
// every prime factor is in range; workspace: M complex (even), 2 n complex (odd)
static bool ft_native_plan(int64_t n, FtPlan* pl) {
  if (n < 2 || n > INT32_MAX) return false;
  if (DPZ_KNOB_INT(FFT_LIB, 0) != 0) return false;  // diagnostic build: hipFFT (A/B)
  return ft_make_plan(n % 2 == 0 ? n / 2 : n, pl);
}

static int64_t ft_native_ws(int64_t n) {
  // even: M complex (aligned up to 256 inside); odd: two n-complex buffers, the second aligned up
  // to 256 past the first + 64 (ft_align): 16 n + 64 + 2 * 255 bounds both
  return n % 2 == 0 ? (n / 2) * 8 + 256 : 2 * n * 8 + 1024;
}

static float2* ft_align(void* ws, size_t off) {
  const uintptr_t u = (reinterpret_cast<uintptr_t>(ws) + off + 255) & ~uintptr_t(255);
  return reinterpret_cast<float2*>(u);
}

static int ft_rfft_native(const FtPlan& pl, const float* x, int64_t n, float2* out, void* ws,
                          size_t ws_bytes, hipStream_t st) {
  if ((int64_t)ws_bytes < ft_native_ws(n) || !ws) return DPZ_ERR_WORKSPACE;
  FtTw tw;
  const int rc = ft_tables((uint32_t)n, &tw);
  if (rc != DPZ_OK) return rc;
  if (n % 2 == 0) {
    const int64_t M = n / 2;
    float2* w = ft_align(ws, 0);
    const float2* z = reinterpret_cast<const float2*>(x);
    // the pairing inside the last pass (DPZ_FFT_POST_FUSED=1, diagnostic build): bit-identical and
    // no faster on MI355X (11 M rfft 168.3 vs 169.1 us, 25 M 368.3 vs 358.4 with the separate
    // pass, profiles/r06_fft_post_ab.jsonl: the mirrored columns' descending stores cost what the
    // pass saves), so the separate pass stays the default
    bool paired = DPZ_KNOB_INT(FFT_POST_FUSED, 0) != 0;
    if (pl.npass > 0) {
      const int r2 = ft_run(pl, tw, false, z, nullptr, 0, out, nullptr, 0, 1.0f, 0, w, out, st,
                            &paired);
      if (r2 != DPZ_OK) return r2;
      z = out;
    } else {
      paired = false;
    }
    if (paired) return DPZ_OK;
    DPZ_TIMED(DPZ_KT_FFT, st, ft_r2c_post_kernel<<<grid_for(M / 2 + 1), 256, 0, st>>>(z, out, M, tw));
    return DPZ_OK;
  }
  float2* a = ft_align(ws, 0);
  float2* b = ft_align(ws, (size_t)n * 8 + 64);
  return ft_run(pl, tw, false, nullptr, x, 1, out, nullptr, 3, 1.0f, n / 2 + 1, a, b, st);
}

static int ft_irfft_native(const FtPlan& pl, float2* coeffs, int64_t n, float* out, void* ws,
                           size_t ws_bytes, hipStream_t st) {
  if ((int64_t)ws_bytes < ft_native_ws(n) || !ws) return DPZ_ERR_WORKSPACE;
  FtTw tw;
  const int rc = ft_tables((uint32_t)n, &tw);
  if (rc != DPZ_OK) return rc;
  const float sc = 1.0f / (float)n;
  if (n % 2 == 0) {
    const int64_t M = n / 2;
    float2* w = ft_align(ws, 0);
    float2* xo = reinterpret_cast<float2*>(out);
    // the inverse DFT_M into out, its first pass forming Z[k] from X[k] and X[M - k] as it loads
    // (load mode 3: no separate pairing pass; the coefficients are only read)
    if (pl.npass == 0) {
      DPZ_TIMED(DPZ_KT_FFT, st, ft_c2r_pre_kernel<<<grid_for(M / 2 + 1), 256, 0, st>>>(
                                    coeffs, xo, M, tw, sc));
      return DPZ_OK;
    }
    if (DPZ_KNOB_INT(FFT_PAIR_FUSED, 1) == 0) {  // diagnostic build: the separate pairing pass (A/B)
      DPZ_TIMED(DPZ_KT_FFT, st, ft_c2r_pre_kernel<<<grid_for(M / 2 + 1), 256, 0, st>>>(
                                    coeffs, coeffs, M, tw, 1.0f));
      return ft_run(pl, tw, true, coeffs, nullptr, 0, xo, nullptr, 1, sc, 0, w, xo, st);
    }
    return ft_run(pl, tw, true, coeffs, nullptr, 3, xo, nullptr, 1, sc, M, w, xo, st);
  }
  float2* a = ft_align(ws, 0);
  float2* b = ft_align(ws, (size_t)n * 8 + 64);
  return ft_run(pl, tw, true, coeffs, nullptr, 2, nullptr, out, 2, sc, n, a, b, st);
}

// ---- plan cache -------------------------------------------------------------------------------
struct FftPlan {
  hipfftHandle h;
  size_t work;
};

static std::mutex g_fft_mu;
static std::map<std::tuple<int, int64_t, int>, FftPlan> g_fft_plans;

// direction 0 = R2C (n reals -> n/2 + 1 complex), 1 = C2R (n/2 + 1 complex -> n reals)
static int fft_plan(int64_t n, int dir, FftPlan* out) {
  int dev = 0;
  DPZ_HIP_TRY(hipGetDevice(&dev));
  const auto key = std::make_tuple(dev, n, dir);
  auto it = g_fft_plans.find(key);
  if (it != g_fft_plans.end()) {
    *out = it->second;
    return DPZ_OK;
  }
  FftPlan p{};
  if (hipfftCreate(&p.h) != HIPFFT_SUCCESS) return DPZ_ERR_INTERNAL;
  if (hipfftSetAutoAllocation(p.h, 0) != HIPFFT_SUCCESS ||
      hipfftMakePlan1d(p.h, (int)n, dir == 0 ? HIPFFT_R2C : HIPFFT_C2R, 1, &p.work) !=
          HIPFFT_SUCCESS) {
    hipfftDestroy(p.h);
    return DPZ_ERR_INTERNAL;
  }
  g_fft_plans.emplace(key, p);
  *out = p;
  return DPZ_OK;
}

static int fft_exec(int64_t n, int dir, void* in, void* out, void* ws, size_t ws_bytes,
                    hipStream_t st) {
  if (n < 2 || n > INT32_MAX) return DPZ_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> lock(g_fft_mu);
  FftPlan p;
  const int rc = fft_plan(n, dir, &p);
  if (rc != DPZ_OK) return rc;
  if (p.work > 0 && (!ws || ws_bytes < p.work)) return DPZ_ERR_WORKSPACE;
  if (hipfftSetWorkArea(p.h, p.work > 0 ? ws : nullptr) != HIPFFT_SUCCESS ||
      hipfftSetStream(p.h, st) != HIPFFT_SUCCESS)
    return DPZ_ERR_INTERNAL;
  const hipfftResult r =
      dir == 0 ? hipfftExecR2C(p.h, static_cast<hipfftReal*>(in), static_cast<hipfftComplex*>(out))
               : hipfftExecC2R(p.h, static_cast<hipfftComplex*>(in), static_cast<hipfftReal*>(out));
  return r == HIPFFT_SUCCESS ? DPZ_OK : DPZ_ERR_INTERNAL;
}

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_fft_workspace_bytes(int64_t n) {
  if (n < 2 || n > INT32_MAX) return -1;
  FtPlan pl;
  if (ft_native_plan(n, &pl)) return ft_native_ws(n);
  std::lock_guard<std::mutex> lock(g_fft_mu);
  FftPlan a, b;
  if (fft_plan(n, 0, &a) != DPZ_OK || fft_plan(n, 1, &b) != DPZ_OK) return -1;
  const size_t w = a.work > b.work ? a.work : b.work;
  return (int64_t)(w > 0 ? w : 0);
}

extern "C" int dpz_fft_native(int64_t n) {
  FtPlan pl;
  return ft_native_plan(n, &pl) ? 1 : 0;
}

extern "C" int dpz_rfft(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                        dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!x || !out || n < 2) return DPZ_ERR_ARG;
  FtPlan pl;
  if (ft_native_plan(n, &pl))
    return ft_rfft_native(pl, x, n, reinterpret_cast<float2*>(out), ws, ws_bytes, st);
  // out-of-place R2C leaves its input untouched
  return fft_exec(n, 0, const_cast<float*>(x), out, ws, ws_bytes, st);
}

extern "C" int dpz_irfft(float* coeffs, int64_t n, float* out, void* ws, size_t ws_bytes,
                         dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!coeffs || !out || n < 2) return DPZ_ERR_ARG;
  FtPlan pl;
  if (ft_native_plan(n, &pl))
    return ft_irfft_native(pl, reinterpret_cast<float2*>(coeffs), n, out, ws, ws_bytes, st);
  const int rc = fft_exec(n, 1, coeffs, out, ws, ws_bytes, st);
  if (rc != DPZ_OK) return rc;
  DPZ_TIMED(DPZ_KT_FFT_SCALE, st, scale_kernel<<<grid_for(n), 256, 0, st>>>(out, n, 1.0f / (float)n));
  return DPZ_OK;
}

extern "C" int dpz_cplx_key(const float* change, float* acc, int acc_mode, int64_t m, float* key,
                            dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (m < 0 || (m > 0 && (!change || !key))) return DPZ_ERR_ARG;
  if (acc_mode != DPZ_ACC_NONE && !acc) return DPZ_ERR_ARG;
  if (m == 0) return DPZ_OK;
  const float2* c = reinterpret_cast<const float2*>(change);
  float2* a = reinterpret_cast<float2*>(acc);
  switch (acc_mode) {
    case DPZ_ACC_NONE:
      DPZ_TIMED(DPZ_KT_CPLX, st, cplx_key_kernel<DPZ_ACC_NONE><<<grid_for(m), 256, 0, st>>>(c, a, m, key));
      break;
    case DPZ_ACC_ACCUMULATE:
      DPZ_TIMED(DPZ_KT_CPLX, st, cplx_key_kernel<DPZ_ACC_ACCUMULATE><<<grid_for(m), 256, 0, st>>>(c, a, m, key));
      break;
    case DPZ_ACC_ADD:
      DPZ_TIMED(DPZ_KT_CPLX, st, cplx_key_kernel<DPZ_ACC_ADD><<<grid_for(m), 256, 0, st>>>(c, a, m, key));
      break;
    default:
      return DPZ_ERR_ARG;
  }
  return DPZ_OK;
}

extern "C" int dpz_cplx_gather(const float* src, int64_t m, const int32_t* idx, int64_t k,
                               float* out, float* acc, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (m < 0 || k < 0 || (k > 0 && (!src || !idx || !out))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  DPZ_TIMED(DPZ_KT_CPLX, st,
            cplx_gather_kernel<<<grid_for(k), 256, 0, st>>>(
                reinterpret_cast<const float2*>(src), m, idx, k, reinterpret_cast<float2*>(out),
                reinterpret_cast<float2*>(acc)));
  return DPZ_OK;
}

extern "C" int dpz_cplx_pair_indices(const int32_t* idx, int64_t k, int32_t* pair,
                                     dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (k < 0 || (k > 0 && (!idx || !pair))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  if (!aligned16(pair) && (reinterpret_cast<uintptr_t>(pair) & 7u)) return DPZ_ERR_ARG;
  DPZ_TIMED(DPZ_KT_CPLX, st, cplx_pair_idx_kernel<<<grid_for(k), 256, 0, st>>>(idx, k, pair));
  return DPZ_OK;
}
