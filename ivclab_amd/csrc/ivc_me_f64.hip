// ivc_me_f64.hip — the pruned float64 full search (MotionCompensator.compute_motion_vector on
// the non-integer float64 luma VideoCodec passes it, ivclab/video/videocodec.py:38,52 ->
// ivclab/video/motion.py:46-48): a float32 bound phase with a rigorous error bound, then the
// reference's float64 SSD only for the candidates the bound cannot exclude.  Its own
// translation unit: built with -fno-slp-vectorize (ivclab_amd/build.py), because the SLP
// vectoriser pairs the bound phase's float32 operations into v_pk_* forms whose operand
// pairing splits the window's 16-byte LDS reads into conflicting 12- and 4-byte ones.
#include "ivc_internal.h"

namespace ivc {

// ---------------------------------------------------------------- pruned float64 search --
// The same result as me_flt_kernel<double, SR> (NumPy's float64 SSD in its pairwise order, first
// strict minimum), in two phases (VideoCodec's search runs on non-integer float64 luma,
// videocodec.py:38,52 -> motion.py:46-48):
//
// 1. Bound.  Every candidate's SSD is computed in float32 from float32 copies of the pixels
//    (v_sub + v_fma per candidate-pixel, against 3 float64 operations at half the rate).  With
//    u = 2^-24, u' = u (1 + u), M >= max|a| + max|b| over the round's pixels, D* the exact
//    real SSD and A the float32 one (any summation order of 64 FMAs):
//      |d' - d| <= u'(|a| + |b|) + u|d| <= u'(M + |d|)            (two conversions, one sub)
//      sum |d'^2 - d^2| <= 16 u' M sqrt(D*) + 2 u' D* + 256 u'^2 M^2  (Cauchy-Schwarz)
//      |A - sum d'^2| <= g64 sum d'^2,  g64 = 64 u / (1 - 64 u)       (64 rounded FMAs)
//    so |A - D*| <= B(D*) = al D* + be sqrt(D*) + g0 with al = g64 + 2u'(1 + g64) < 3.94e-6,
//    be = 16 u'(1 + g64) M < 9.6e-7 M, g0 = 256 u'^2 (1 + g64) M^2 < 9.2e-13 M^2; the kernel uses
//    al = 2^-17, be = 2^-19 M, g0 = 2^-38 M^2 + 2^-100 (the last: float32 results flushed
//    below 2^-126).  The reference's S (float64, 13 roundings on any path) is within
//    (1 +- 2^-40) of D*.  For the block's least A, Amin: D* <= X^2 with
//    X = (be + sqrt(be^2 + 4 (1 - al)(g0 + Amin))) / (2 (1 - al)) (the root of
//    (1 - al) x^2 - be x - (g0 + Amin)), so min S <= V = X^2 (1 + 2^-38); a candidate with
//    S <= min S has D* <= V, hence A <= T = V + B(V).  T is formed in float64 with a 2^-30
//    margin and rounded up to float32.
// 2. Exact.  The candidates with A <= T (the block's least-A candidate always among them) are
//    listed in LDS; groups of 8 lanes evaluate them in the reference's order from the frames
//    in global memory (lane j: column j's sum down the rows, then the pairwise tree by xor
//    shuffles — float64 addition is commutative, so every lane of the tree holds the same
//    bits), and the block's (S, raster index) minimum is taken as in me_flt_kernel.
// A round whose pixels are not all finite with |x| <= 2^24 and (x == 0 or |x| >= 2^-60) (where
// the bound's assumptions fail: NaN, inf, float32 overflow or underflow), or whose list
// overflows (e.g. flat content where every candidate ties), is deferred: its index is appended
// to a device list and me_flt_kernel searches the listed rounds afterwards.  Rounds are the
// same NBR-block segments of a block row in both kernels.
constexpr int F64P_CAP = 768;
#ifndef IVC_F64P_WAVES
#define IVC_F64P_WAVES 6   // waves per SIMD the pruned kernel is built for (3 workgroups per CU)
#endif                               // listed candidates per round

template <int SR> struct F64pGeom {
  typedef FltGeom<double, SR> G;
  static constexpr int N = G::N, NBR = G::NBR, WR = G::WR, WC = G::WC;
  // window column pitch (float32): >= WR, a multiple of 4 with an odd quotient, so the 16
  // lanes of a ds_read_b128 quarter-wave reading consecutive columns start on distinct
  // 4-dword bank groups (64 banks)
  static constexpr int P = ((WR + 3) / 4 % 2 == 1) ? (WR + 3) / 4 * 4 : (WR + 3) / 4 * 4 + 4;
  static_assert(NBR * N <= FLT_WG && P % 4 == 0 && (P / 4) % 2 == 1, "pruned geometry");
};

__device__ __forceinline__ float f64p_threshold(float amin, float m) {
  const double A = amin, M = (double)m * (1.0 + 0x1p-20);
  const double al = 0x1p-17, be = 0x1p-19 * M, g0 = 0x1p-38 * M * M + 0x1p-100;
  const double X = (be + sqrt(be * be + 4.0 * (1.0 - al) * (g0 + A))) / (2.0 * (1.0 - al));
  const double V = X * X * (1.0 + 0x1p-38);
  const double T = (V + al * V + be * sqrt(V) + g0) * (1.0 + 0x1p-30);
  float t = (float)T;
  if ((double)t < T) t = __uint_as_float(__float_as_uint(t) + 1u);   // up (t >= 0)
  return t;
}

// The same bound formed in float32: every operation is a sum, product, quotient by a constant
// or square root of non-negative values (T increases with each of them), and each rounds to
// nearest within 2^-24 relative, so the ~12 roundings leave the result at most 12 * 2^-24
// below the exact T; multiplying by (1 + 2^-18) and stepping one ulp up covers that, the
// 2^-38 and 2^-30 margins above, and v_sqrt_f32's error (< 1 ulp).
__device__ __forceinline__ float f64p_threshold32(float amin, float m) {
  const float M = m * (1.0f + 0x1p-20f);
  const float al = 0x1p-17f, be = 0x1p-19f * M, g0 = 0x1p-38f * (M * M) + 0x1p-100f;
  const float X = (be + __builtin_sqrtf(be * be + (4.0f - 0x1p-15f) * (g0 + amin))) *
                  (1.0f / (2.0f - 0x1p-16f));
  const float V = X * X;
  const float T = (V + al * V + be * __builtin_sqrtf(V) + g0) * (1.0f + 0x1p-18f);
  return __uint_as_float(__float_as_uint(T) + 1u);
}
#ifndef IVC_F64P_T32
#define IVC_F64P_T32 1
#endif
#ifndef IVC_F64P_MASK
#define IVC_F64P_MASK 1
#endif
#ifndef IVC_F64P_PREFETCH
#define IVC_F64P_PREFETCH 0
#endif

template <int SR>
__global__ __launch_bounds__(FLT_WG, IVC_F64P_WAVES) void me_f64p_kernel(const double* __restrict__ ref,
                                                            const double* __restrict__ cur,
                                                            int64_t nframes, int H, int W,
                                                            int64_t* __restrict__ mv,
                                                            uint32_t* __restrict__ defer,
                                                            int defer_all) {
  typedef F64pGeom<SR> G;
  constexpr int n = G::N, nbr = G::NBR, WR = G::WR, WC = G::WC, P = G::P;
  __shared__ __attribute__((aligned(16))) float winT[WC * P];     // [column][row]
  __shared__ __attribute__((aligned(16))) float cbT[nbr * 64];    // [block][v][u]
  __shared__ uint32_t ent[F64P_CAP];                              // block << 16 | raster index
  __shared__ double sval[F64P_CAP];
  __shared__ unsigned long long kmin[nbr];
  __shared__ uint32_t amin[nbr], imin[nbr];
  __shared__ uint32_t nsurv, bad, mw, mb;
  const int h = H / 8, w = W / 8;
  const int segs = (w + nbr - 1) / nbr;
  const int64_t rounds = nframes * h * segs;
  constexpr int NWI = (WR * WC + FLT_WG - 1) / FLT_WG, NBI = (nbr * 64 + FLT_WG - 1) / FLT_WG;
  // the round's window and blocks as float64, every load of the thread issued before the first
  // use (one memory latency per round)
  auto load_round = [&](int64_t rr, int tid, double (&wv)[NWI], double (&bv)[NBI]) {
    const bool ex = rr < rounds;
    const int64_t f = ex ? rr / ((int64_t)h * segs) : 0;
    const int rem = ex ? (int)(rr - f * h * segs) : 0, by = rem / segs, bx0 = (rem - by * segs) * nbr;
    const int nb = w - bx0 < nbr ? w - bx0 : nbr;
    const double* rf = ref + f * (int64_t)H * W;
    const double* cf = cur + f * (int64_t)H * W;
    const int y0 = 8 * by - SR, x0 = 8 * bx0 - SR, wc = nb * 8 + 2 * SR;
#pragma unroll
    for (int j = 0; j < NWI; ++j) {
      const int i = tid + j * FLT_WG;
      const int xx = i / WR, yy = i - xx * WR, gy = y0 + yy, gx = x0 + xx;
      wv[j] = (ex && i < WR * wc && gy >= 0 && gy < H && gx >= 0 && gx < W) ? rf[(int64_t)gy * W + gx] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < NBI; ++j) {
      const int i = tid + j * FLT_WG;
      const int b = i >> 6, u = (i >> 3) & 7, v = i & 7;
      bv[j] = ex && i < nb * 64 ? cf[(int64_t)(8 * by + u) * W + 8 * (bx0 + b) + v] : 0.0;
    }
  };
  double wv[NWI], bv[NBI];
  if (IVC_F64P_PREFETCH) load_round(blockIdx.x, threadIdx.x, wv, bv);
  for (int64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    // (opaque per round: the thread's index constants are formed in the loop instead of being
    // hoisted out of it, where they stay live — and spill — through the search)
    int tid = threadIdx.x;
    __asm__ volatile("" : "+v"(tid));
    const int sb = tid / n, se = tid - sb * n;                    // block of the round, column
    const int64_t f = r / ((int64_t)h * segs);
    const int rem = (int)(r - f * h * segs), by = rem / segs, bx0 = (rem - by * segs) * nbr;
    const int nb = w - bx0 < nbr ? w - bx0 : nbr;
    const double* rf = ref + f * (int64_t)H * W;
    const double* cf = cur + f * (int64_t)H * W;
    const int wc = nb * 8 + 2 * SR;
    lds_barrier();                                  // the previous round's LDS reads are done
    if (tid == 0) {
      nsurv = 0;
      bad = 0;
      mw = 0;
      mb = 0;
    }
    if (tid < nbr) {
      amin[tid] = ~0u;
      kmin[tid] = ~0ull;
      imin[tid] = ~0u;
    }
    // stage the window (column-major float32, zeros outside the frame) and the blocks, checking
    // the bound's assumptions and taking max |x| on the way
    bool badl = false;
    float mwl = 0.f, mbl = 0.f;
    if (!IVC_F64P_PREFETCH) load_round(r, tid, wv, bv);
#pragma unroll
    for (int j = 0; j < NWI; ++j) {
      const int i = tid + j * FLT_WG;
      const int xx = i / WR, yy = i - xx * WR;
      const double av = fabs(wv[j]);
      badl |= !(av <= 0x1p24) || (av != 0.0 && av < 0x1p-60);
      const float fv = (float)wv[j];
      mwl = fmaxf(mwl, fabsf(fv));
      if (i < WR * wc) winT[xx * P + yy] = fv;
    }
#pragma unroll
    for (int j = 0; j < NBI; ++j) {
      const int i = tid + j * FLT_WG;
      const int b = i >> 6, u = (i >> 3) & 7, v = i & 7;
      const double ax = fabs(bv[j]);
      badl |= !(ax <= 0x1p24) || (ax != 0.0 && ax < 0x1p-60);
      const float fx = (float)bv[j];
      mbl = fmaxf(mbl, fabsf(fx));
      if (i < nb * 64) cbT[b * 64 + v * 8 + u] = fx;
    }
    // (IVC_F64P_PREFETCH: the next round's loads fly during this round's search)
    if (IVC_F64P_PREFETCH) load_round(r + gridDim.x, tid, wv, bv);
    lds_barrier();                                  // (the resets above are visible)
    if (badl) atomicOr(&bad, 1u);
    atomicMax(&mw, __float_as_uint(mwl));
    atomicMax(&mb, __float_as_uint(mbl));
    // phase 1: float32 SSD of the thread's column of candidates, all dy at once
    const int rx = 8 * (bx0 + sb) + se - SR;
    const bool col = sb < nb && rx >= 0 && rx + 8 <= W;
    const int ky0 = max(0, SR - 8 * by), ky1 = min(n, H - 8 - 8 * by + SR + 1);   // valid dy
    float acc[n];
#pragma unroll
    for (int k = 0; k < n; ++k) acc[k] = 0.f;
    float m = __builtin_inff();                     // the lane's least A over its valid dy
    if (col) {
      const float* cb = cbT + sb * 64;
      const float* wcol = winT + (sb * 8 + se) * P;
#pragma unroll 1
      for (int v = 0; v < 8; ++v) {
        // window column e + v streamed row by row: row r serves candidates k = r - u
        float cv[8];
#pragma unroll
        for (int u = 0; u < 8; u += 4) {
          const float4 q = *reinterpret_cast<const float4*>(cb + v * 8 + u);
          cv[u] = q.x; cv[u + 1] = q.y; cv[u + 2] = q.z; cv[u + 3] = q.w;
        }
        // the next group of 4 rows is read one group ahead (its LDS latency under this group's
        // 64 operations); the 8 differences of a row are formed before their 8 FMAs
        float4 qn = *reinterpret_cast<const float4*>(wcol + v * P);
#pragma unroll
        for (int r4 = 0; r4 < WR; r4 += 4) {
          const float4 q = qn;
          if (r4 + 4 < WR) qn = *reinterpret_cast<const float4*>(wcol + v * P + r4 + 4);
          // (no later LDS read moves above this point: the compiler would hoist the whole
          // column's reads and spill)
          __asm__ volatile("" ::: "memory");
          const float wq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            float d[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = cv[u] - wq[t];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int k = r4 + t - u;
              if (k >= 0 && k < n) acc[k] = __builtin_fmaf(d[u], d[u], acc[k]);
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < n; ++k)
        if (k >= ky0 && k < ky1) m = fminf(m, acc[k]);
      if (m != __builtin_inff()) atomicMin(&amin[sb], __float_as_uint(m));
    }
    lds_barrier();
    if (bad == 0u && col) {
      const float t = IVC_F64P_T32 ? f64p_threshold32(__uint_as_float(amin[sb]),
                                                      __uint_as_float(mw) + __uint_as_float(mb))
                                   : f64p_threshold(__uint_as_float(amin[sb]),
                                                    __uint_as_float(mw) + __uint_as_float(mb));
#if IVC_F64P_MASK
      // only lanes whose least A is within T have survivors: their dy as a bit mask, then one
      // append per set bit (usually one)
      if (m <= t) {
        uint64_t mk = 0;
#pragma unroll
        for (int k = 0; k < n; ++k)
          mk |= (uint64_t)(k >= ky0 && k < ky1 && acc[k] <= t) << k;
        while (mk) {
          const int k = __builtin_ctzll(mk);
          mk &= mk - 1;
          const uint32_t slot = atomicAdd(&nsurv, 1u);
          if (slot < (uint32_t)F64P_CAP) ent[slot] = ((uint32_t)sb << 16) | (uint32_t)(k * n + se);
        }
      }
#else
#pragma unroll
      for (int k = 0; k < n; ++k)
        if (k >= ky0 && k < ky1 && acc[k] <= t) {
          const uint32_t slot = atomicAdd(&nsurv, 1u);
          if (slot < (uint32_t)F64P_CAP) ent[slot] = ((uint32_t)sb << 16) | (uint32_t)(k * n + se);
        }
#endif
    }
    lds_barrier();
    const uint32_t ns = nsurv;
    if (bad != 0u || ns > (uint32_t)F64P_CAP || defer_all) {   // (workgroup-uniform) deferred
      if (tid == 0) {
        const uint32_t k = atomicAdd(defer, 1u);
        defer[1 + k] = (uint32_t)r;
      }
      continue;
    }
    // phase 2: the listed candidates in the reference's order, 8 lanes each
    const int lj = tid & 7;
    for (uint32_t e = (uint32_t)(tid >> 3); e < ns; e += FLT_WG / 8) {
      const uint32_t en = ent[e];
      const int b = (int)(en >> 16), c = (int)(en & 0xffffu);
      const int dy = c / n - SR, dx = c - (c / n) * n - SR;
      const double* R = rf + (int64_t)(8 * by + dy) * W + 8 * (bx0 + b) + dx + lj;
      const double* B = cf + (int64_t)(8 * by) * W + 8 * (bx0 + b) + lj;
      double bv[8], rv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        bv[u] = B[(int64_t)u * W];
        rv[u] = R[(int64_t)u * W];
      }
      double d = bv[0] - rv[0];
      double s = d * d;
#pragma unroll
      for (int u = 1; u < 8; ++u) {
        d = bv[u] - rv[u];
        s = s + d * d;
      }
      s = s + __shfl_xor(s, 1, 8);                  // (c0 + c1) ...
      s = s + __shfl_xor(s, 2, 8);                  // ((c0 + c1) + (c2 + c3)) ...
      s = s + __shfl_xor(s, 4, 8);
      if (lj == 0) {
        sval[e] = s;
        if (s < (double)INFINITY) atomicMin(&kmin[b], (unsigned long long)__double_as_longlong(s));
      }
    }
    lds_barrier();
    for (uint32_t e = (uint32_t)tid; e < ns; e += FLT_WG) {
      const uint32_t en = ent[e];
      const int b = (int)(en >> 16);
      if ((unsigned long long)__double_as_longlong(sval[e]) == kmin[b]) atomicMin(&imin[b], en & 0xffffu);
    }
    lds_barrier();
    if (tid < nb)
      mv[(f * h + by) * w + bx0 + tid] = imin[tid] == ~0u ? (int64_t)SR * n + SR : (int64_t)imin[tid];
  }
}

template <int SR>
static void launch_sr(const double* ref, const double* cur, int64_t nf, int H, int W, int64_t* mv,
                      uint32_t* defer, int defer_all, hipStream_t s) {
  typedef F64pGeom<SR> G;
  const int h = H / 8, w = W / 8;
  const int64_t rounds = nf * h * ((w + G::NBR - 1) / G::NBR);
  int64_t grid = (int64_t)resident_grid_ptr(reinterpret_cast<const void*>(me_f64p_kernel<SR>), rounds);
  if (grid > rounds) grid = rounds;
  if (grid < 1) grid = 1;
  me_f64p_kernel<SR><<<(unsigned)grid, FLT_WG, 0, s>>>(ref, cur, nf, H, W, mv, defer, defer_all);
}

bool launch_me_f64p(int sr, const double* ref, const double* cur, int64_t nf, int H, int W,
                    int64_t* mv, uint32_t* defer, int defer_all, hipStream_t s) {
  switch (sr) {
    case 4: launch_sr<4>(ref, cur, nf, H, W, mv, defer, defer_all, s); return true;
    case 8: launch_sr<8>(ref, cur, nf, H, W, mv, defer, defer_all, s); return true;
    case 16: launch_sr<16>(ref, cur, nf, H, W, mv, defer, defer_all, s); return true;
    default: return false;
  }
}

}  // namespace ivc
