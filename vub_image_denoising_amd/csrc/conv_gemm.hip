// Implicit-GEMM convolution for gfx950 (MFMA), NHWC activations.
//
//   out[m, j] = epilogue( sum_k A[m, k] * P[j, k] )
//
// GEMM row m is a pixel of the row grid (n, h, w); K = taps * cin with
// k = tap * cin + ci, so every 16-byte unit a lane gathers (8 bf16 / 4 fp32
// channels of one source pixel) is contiguous in NHWC memory.  The tap decides
// the source pixel (RDN_G_CONV3: 3x3 pad 1; RDN_G_S2: 2x2 stride 2; RDN_G_PIX:
// same pixel).  P is the packed weight operand [rows][kp] (k contiguous).
//
// One kernel serves the 3x3 convs of every block (Unet_model.py:48-49,60-61,
// 72-75,35), the 2x2/s2 down-sampling conv (:26), the 2x2/s2 transposed conv
// (:36, as a per-pixel GEMM with a depth-to-space scatter epilogue) and the
// input gradients of all three (the same three shapes with repacked weights).
//
// Tiling: 256 threads = 4 waves; block tile BM x BN; K staged through LDS in
// steps of 8 units (128 B per row), double buffered with a register prefetch
// of the next stage.  bf16: v_mfma_f32_16x16x32_bf16, fp32: v_mfma_f32_16x16x4_f32
// (exact fp32, the mode parity is checked in).
#include "conv3_tile.h"

#include <cstdlib>

namespace {

constexpr int NT = 256;
constexpr int U = 8;                 // 16-byte units per LDS row per stage
constexpr int ROWB = U * 16 + 32;    // padded LDS row: 160 B = 10 slots, conflict-free ds_read_b128

template <int GATHER> struct Taps;
template <> struct Taps<RDN_G_CONV3> { static constexpr int N = 9; };
template <> struct Taps<RDN_G_S2> { static constexpr int N = 4; };
template <> struct Taps<RDN_G_PIX> { static constexpr int N = 1; };

// SPLIT (rdn_conv_fwd_splitk): block layer blockIdx.z walks K stages
// [z * s_per, (z + 1) * s_per) only and stores its raw fp32 tile to ws[z][m][ncols]
template <typename T, int BM, int BN, int WMW, int GATHER, bool SPLIT = false>
__global__ __launch_bounds__(NT) void conv_gemm_kernel(rdn_conv_desc d, FastDiv fd_w, FastDiv fd_hw, int s_per = 0,
                                                       float* __restrict__ ws = nullptr) {
  constexpr int VEC = TypeInfo<T>::VEC;
  constexpr int SK = U * VEC;
  constexpr int WNW = 4 / WMW;
  constexpr int WTM = BM / WMW, WTN = BN / WNW;
  constexpr int MT = WTM / 16, NTL = WTN / 16;
  constexpr int A_UNITS = BM * U, B_UNITS = BN * U;
  constexpr int A_IT = (A_UNITS + NT - 1) / NT, B_IT = (B_UNITS + NT - 1) / NT;
  constexpr int TAPS = Taps<GATHER>::N;
  static_assert(MT >= 1 && NTL >= 1, "tile");

  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * (BM + BN) * ROWB];
#define ldsA(b) (lds + (b) * (BM * ROWB))
#define ldsB(b) (lds + 2 * BM * ROWB + (b) * (BN * ROWB))

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WMW, wn = wave / WMW;
  const int64_t M = (int64_t)d.n * d.h * d.w;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ku = tid & (U - 1);
  const T* __restrict__ X = (const T*)d.x;
  const T* __restrict__ WP = (const T*)d.wp;

  // ---- per-thread A rows (fixed over the K loop)
  int a_y[A_IT], a_x[A_IT];
  int64_t a_base[A_IT];
  bool a_ok[A_IT];
#pragma unroll
  for (int r = 0; r < A_IT; ++r) {
    const int u = tid + r * NT;
    const int64_t m = m0 + (u >> 3);
    a_ok[r] = (u < A_UNITS) && (m < M);
    const uint32_t mm = a_ok[r] ? (uint32_t)m : 0u;
    const uint32_t nimg = fdiv(mm, fd_hw);
    const uint32_t rem = mm - nimg * (uint32_t)(d.h * d.w);
    const uint32_t y = fdiv(rem, fd_w);
    const uint32_t x = rem - y * (uint32_t)d.w;
    a_y[r] = (int)y;
    a_x[r] = (int)x;
    // pixel part only; the channel part (rdn_coff) is added per K stage
    if (GATHER == RDN_G_S2)
      a_base[r] = (((int64_t)nimg * d.hin + 2 * y) * d.win + 2 * x) * d.x_ps;
    else
      a_base[r] = (((int64_t)nimg * d.hin + y) * d.win + x) * d.x_ps;
  }

  const int cin = d.cin;
  const int ktot = TAPS * cin;
  const int s_lo = SPLIT ? (int)blockIdx.z * s_per : 0;
  const int nst = SPLIT ? min((ktot + SK - 1) / SK, s_lo + s_per) : (ktot + SK - 1) / SK;
  int tap = (s_lo * SK + ku * VEC) / cin, ci = (s_lo * SK + ku * VEC) - tap * cin;

  u32x4 ra[A_IT], rb[B_IT];

  auto load_stage = [&](int s) {
    const int64_t cf = rdn_coff(d.x_c0 + ci, d.x_ps, d.x_pl);   // this thread's channel unit
#pragma unroll
    for (int r = 0; r < A_IT; ++r) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (a_ok[r] && tap < TAPS) {
        int64_t off;
        bool ok = true;
        if (GATHER == RDN_G_CONV3) {
          const int dy = tap / 3 - 1, dx = tap % 3 - 1;
          const int ys = a_y[r] + dy, xs = a_x[r] + dx;
          ok = (ys >= 0) && (ys < d.hin) && (xs >= 0) && (xs < d.win);
          off = a_base[r] + ((int64_t)dy * d.win + dx) * d.x_ps + cf;
        } else if (GATHER == RDN_G_S2) {
          off = a_base[r] + ((int64_t)(tap >> 1) * d.win + (tap & 1)) * d.x_ps + cf;
        } else {
          off = a_base[r] + cf;
        }
        if (ok) v = *(const u32x4*)(X + off);
      }
      ra[r] = v;
    }
#pragma unroll
    for (int r = 0; r < B_IT; ++r) {
      const int u = tid + r * NT;
      if (u < B_UNITS) rb[r] = *(const u32x4*)(WP + (int64_t)(n0 + (u >> 3)) * d.kp + (int64_t)s * SK + ku * VEC);
    }
    ci += SK;
    while (ci >= cin) { ci -= cin; ++tap; }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int r = 0; r < A_IT; ++r) {
      const int u = tid + r * NT;
      if (u < A_UNITS) *(u32x4*)(ldsA(buf) + (u >> 3) * ROWB + ku * 16) = ra[r];
    }
#pragma unroll
    for (int r = 0; r < B_IT; ++r) {
      const int u = tid + r * NT;
      if (u < B_UNITS) *(u32x4*)(ldsB(buf) + (u >> 3) * ROWB + ku * 16) = rb[r];
    }
  };

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frag_row = lane & 15, frag_k = (lane >> 4) * 16;

  load_stage(s_lo);
  store_stage(0);
  __syncthreads();
  for (int s = s_lo; s < nst; ++s) {
    const int buf = (s - s_lo) & 1;
    if (s + 1 < nst) load_stage(s + 1);
#pragma unroll
    for (int ks = 0; ks < U / 4; ++ks) {
      u32x4 af[MT], bfr[NTL];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *(const u32x4*)(ldsA(buf) + (wm * WTM + i * 16 + frag_row) * ROWB + ks * 64 + frag_k);
#pragma unroll
      for (int j = 0; j < NTL; ++j)
        bfr[j] = *(const u32x4*)(ldsB(buf) + (wn * WTN + j * 16 + frag_row) * ROWB + ks * 64 + frag_k);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                                __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0, 0, 0);
          } else {
            // whole-vector casts (see rdn_common.h: element bit casts miscompile)
            const f32x4 a4 = __builtin_bit_cast(f32x4, af[i]);
            const f32x4 b4 = __builtin_bit_cast(f32x4, bfr[j]);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], b4[e], acc[i][j], 0, 0, 0);
          }
        }
    }
    if (s + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }

#undef ldsA
#undef ldsB
  // ---- fused epilogue: the fp32 tile goes through LDS (the K loop ended with a
  // barrier) so every global access is a 16-byte unit of VEC channels of one
  // output pixel; with SCATTER2 the unit's columns are VEC channels of one tap
  // (cout % VEC == 0), i.e. one 16-B piece of a depth-to-space output pixel.
  static_assert(BM * (BN + 4) * 4 <= 2 * (BM + BN) * ROWB, "epilogue tile fits the K-loop LDS");
  constexpr int CROW = BN + 4;
  float* const Ct = (float*)lds;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Ct[(wm * WTM + i * 16 + (lane >> 4) * 4 + e) * CROW + wn * WTN + j * 16 + (lane & 15)] = acc[i][j][e];
  __syncthreads();
  if constexpr (SPLIT) {   // raw fp32 slice of the tile: 16-B units of 4 columns (ncols % 4 == 0)
    float* const wz = ws + (int64_t)blockIdx.z * M * d.ncols;
    for (int u = tid; u < BM * (BN / 4); u += NT) {
      const int r = u / (BN / 4), cl = (u - r * (BN / 4)) * 4;
      const int64_t m = m0 + r;
      if (m >= M || n0 + cl >= d.ncols) continue;
      *(f32x4*)(wz + m * d.ncols + n0 + cl) = *(const f32x4*)(Ct + r * CROW + cl);
    }
    return;
  }
  const int flags = d.flags;
  const int H = d.h, W = d.w;
  constexpr int UPR = BN / VEC;
  // fast epilogue: a thread's 16-B column unit is fixed (NT % UPR == 0), so bias /
  // PReLU slope / scatter tap are loaded and decoded once, and every access is a
  // whole 16-B NHWC unit
  static_assert(NT % UPR == 0, "fixed column unit per thread");
  const bool fast = (d.ncols % VEC) == 0 && !(flags & RDN_EPI_OUT_NCHW) && d.out_ps % VEC == 0 &&
                    d.out_c0 % VEC == 0 && d.pre_ps % VEC == 0 &&
                    (!(flags & RDN_EPI_RESID) || (d.res_climit % VEC == 0 && d.res_ps % VEC == 0 &&
                                                  d.res_c0 % VEC == 0));
  if (fast) {
    constexpr int RPI = NT / UPR;              // tile rows per pass
    const int cu = tid % UPR;
    const int col = n0 + cu * VEC;
    if (col >= d.ncols) return;
    int c = col, tp = 0;
    if (flags & RDN_EPI_SCATTER2) { tp = col / d.cout; c = col - tp * d.cout; }
    float eb[VEC], ea[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      eb[q] = (flags & RDN_EPI_BIAS) ? d.bias[c + q] : 0.f;
      ea[q] = (flags & RDN_EPI_PRELU) ? d.alpha[c + q] : 0.f;
    }
    const bool resid = (flags & RDN_EPI_RESID) && c < d.res_climit;
    const int64_t cf_pre = rdn_coff(c, d.pre_ps, d.pre_pl), cf_out = rdn_coff(d.out_c0 + c, d.out_ps, d.out_pl);
    const int64_t cf_res = rdn_coff(d.res_c0 + c, d.res_ps, d.res_pl);
#pragma unroll 2
    for (int r = tid / UPR; r < BM; r += RPI) {
      const int64_t m = m0 + r;
      if (m >= M) break;
      int64_t opix = m;
      if (flags & RDN_EPI_SCATTER2) {
        const int nimg = (int)fdiv((uint32_t)m, fd_hw);
        const int rem = (int)m - nimg * H * W;
        const int y = (int)fdiv((uint32_t)rem, fd_w);
        const int x = rem - y * W;
        opix = ((int64_t)nimg * (2 * H) + 2 * y + (tp >> 1)) * (2 * W) + 2 * x + (tp & 1);
      }
      float v[VEC];
      const float* src = Ct + r * CROW + cu * VEC;
#pragma unroll
      for (int q = 0; q < VEC; q += 4) {
        const f32x4 t4 = *(const f32x4*)(src + q);
        v[q] = t4[0]; v[q + 1] = t4[1]; v[q + 2] = t4[2]; v[q + 3] = t4[3];
      }
      if (flags & RDN_EPI_BIAS) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) v[q] += eb[q];
      }
      if (flags & RDN_EPI_STORE_PRE) *(u32x4*)((T*)d.pre + opix * d.pre_ps + cf_pre) = Unit16<T>::pack(v);
      if (flags & RDN_EPI_PRELU) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) v[q] = v[q] > 0.f ? v[q] : ea[q] * v[q];
      }
      T* const op = (T*)d.out + opix * d.out_ps + cf_out;
      if (resid || (flags & RDN_EPI_ACCUM)) {
        float rv[VEC];
        if (resid) {
          Unit16<T>::unpack(*(const u32x4*)((const T*)d.res + opix * d.res_ps + cf_res), rv);
#pragma unroll
          for (int q = 0; q < VEC; ++q) v[q] += rv[q];
        }
        if (flags & RDN_EPI_ACCUM) {
          Unit16<T>::unpack(*(const u32x4*)op, rv);
#pragma unroll
          for (int q = 0; q < VEC; ++q) v[q] += rv[q];
        }
      }
      *(u32x4*)op = Unit16<T>::pack(v);
    }
    return;
  }
#pragma nounroll
  for (int u = tid; u < BM * UPR; u += NT) {
    const int r = u / UPR, cu = u - r * UPR;
    const int64_t m = m0 + r;
    const int col = n0 + cu * VEC;
    if (m >= M || col >= d.ncols) continue;
    int c = col, tp = 0;
    if (flags & RDN_EPI_SCATTER2) { tp = col / d.cout; c = col - tp * d.cout; }
    int64_t opix = m;
    int nimg = 0, y = 0, x = 0;
    if (flags & (RDN_EPI_SCATTER2 | RDN_EPI_OUT_NCHW)) {
      nimg = (int)fdiv((uint32_t)m, fd_hw);
      const int rem = (int)m - nimg * H * W;
      y = (int)fdiv((uint32_t)rem, fd_w);
      x = rem - y * W;
      if (flags & RDN_EPI_SCATTER2) {
        y = 2 * y + (tp >> 1);
        x = 2 * x + (tp & 1);
        opix = ((int64_t)nimg * (2 * H) + y) * (2 * W) + x;
      }
    }
    float v[VEC];
    const float* src = Ct + r * CROW + cu * VEC;
#pragma unroll
    for (int q = 0; q < VEC; q += 4) {
      const f32x4 t4 = *(const f32x4*)(src + q);
      v[q] = t4[0]; v[q + 1] = t4[1]; v[q + 2] = t4[2]; v[q + 3] = t4[3];
    }
    c3::finish_unit<T>(d, v, c, opix, y, x, nimg, c3::PF_NONE, u32x4{0u, 0u, 0u, 0u});
  }
}

template <typename T, int BM, int BN, int WMW>
int launch_gather(const rdn_conv_desc* d, hipStream_t st, int splits = 0, float* ws = nullptr) {
  const int64_t M = (int64_t)d->n * d->h * d->w;
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((d->ncols + BN - 1) / BN));
  FastDiv fw = make_fastdiv((uint32_t)d->w), fhw = make_fastdiv((uint32_t)(d->h * d->w));
  if (splits > 0) {   // split-K layers (rdn_conv_fwd_splitk): 2x2 / per-pixel gathers only
    constexpr int SK = 8 * TypeInfo<T>::VEC;
    const int taps = d->gather == RDN_G_S2 ? 4 : 1;
    const int nst = (taps * d->cin + SK - 1) / SK, s_per = (nst + splits - 1) / splits;
    grid.z = (unsigned)((nst + s_per - 1) / s_per);
    RDN_PROBE("conv_gemm_kernel<%s,%d,%d,%d,%d,split>", rdn_tname<T>(), BM, BN, WMW, d->gather);
    if (d->gather == RDN_G_S2)
      conv_gemm_kernel<T, BM, BN, WMW, RDN_G_S2, true><<<grid, NT, 0, st>>>(*d, fw, fhw, s_per, ws);
    else
      conv_gemm_kernel<T, BM, BN, WMW, RDN_G_PIX, true><<<grid, NT, 0, st>>>(*d, fw, fhw, s_per, ws);
    return rdn_check_launch("rdn_conv_fwd_splitk(gemm)");
  }
  RDN_PROBE("conv_gemm_kernel<%s,%d,%d,%d,%d>", rdn_tname<T>(), BM, BN, WMW, d->gather);
  switch (d->gather) {
    case RDN_G_CONV3: conv_gemm_kernel<T, BM, BN, WMW, RDN_G_CONV3><<<grid, NT, 0, st>>>(*d, fw, fhw); break;
    case RDN_G_S2: conv_gemm_kernel<T, BM, BN, WMW, RDN_G_S2><<<grid, NT, 0, st>>>(*d, fw, fhw); break;
    default: conv_gemm_kernel<T, BM, BN, WMW, RDN_G_PIX><<<grid, NT, 0, st>>>(*d, fw, fhw); break;
  }
  return rdn_check_launch("rdn_conv_fwd");
}

static int gemm_bn(const rdn_conv_desc* d) {
  return d->bn ? d->bn : d->ncols <= 16 ? 16 : d->ncols <= 32 ? 32 : d->ncols <= 64 ? 64 : 128;
}

template <typename T>
int launch_typed(const rdn_conv_desc* d, hipStream_t st, int splits = 0, float* ws = nullptr) {
  switch (gemm_bn(d)) {
    case 16: return launch_gather<T, 128, 16, 4>(d, st, splits, ws);
    case 32: return launch_gather<T, 128, 32, 4>(d, st, splits, ws);
    case 64: return launch_gather<T, 128, 64, 2>(d, st, splits, ws);
    case 128: return launch_gather<T, 128, 128, 2>(d, st, splits, ws);
  }
  rdn_set_error("rdn_conv_fwd: unsupported bn=%d", gemm_bn(d));
  return RDN_E_ARG;
}

}  // namespace

// A/B switch of conv_pix.hip (RDN_PIX=0: the 2x2 shapes stay on conv_gemm_kernel)
static const bool RDN_PIX = [] {
  const char* e = getenv("RDN_PIX");
  return !(e && e[0] == '0');
}();

extern "C" int rdn_conv_fwd(const rdn_conv_desc* d, void* stream) {
  if (!d || !d->x || !d->wp) { rdn_set_error("rdn_conv_fwd: null descriptor/pointer"); return RDN_E_ARG; }
  const int vec = d->dtype == RDN_BF16 ? 8 : 4;
  if (d->dtype != RDN_F32 && d->dtype != RDN_BF16) { rdn_set_error("rdn_conv_fwd: bad dtype %d", d->dtype); return RDN_E_ARG; }
  if (d->gather < RDN_G_CONV3 || d->gather > RDN_G_PIX) { rdn_set_error("rdn_conv_fwd: bad gather %d", d->gather); return RDN_E_ARG; }
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->cin <= 0 || d->ncols <= 0) {
    rdn_set_error("rdn_conv_fwd: empty shape n=%d h=%d w=%d cin=%d ncols=%d", d->n, d->h, d->w, d->cin, d->ncols);
    return RDN_E_SHAPE;
  }
  if (d->cin % 8 || d->x_ps % vec || d->x_c0 % vec || d->kp % 64 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15)) {
    rdn_set_error("rdn_conv_fwd: alignment (cin=%d x_ps=%lld x_c0=%d kp=%d) must keep 16-byte units", d->cin,
                  (long long)d->x_ps, d->x_c0, d->kp);
    return RDN_E_SHAPE;
  }
  if ((d->x_pl && (d->x_pl < (int64_t)d->n * d->hin * d->win * d->x_ps || rdn_coff(d->x_c0 + d->cin - 1, d->x_ps, d->x_pl) >= (1ll << 31))) ||
      (d->out_pl && d->out_ps % vec) || (d->res_pl && d->res_ps % vec) || (d->gate_pl && d->gate_ps % vec)) {
    rdn_set_error("rdn_conv_fwd: channel-blocked operand needs ps %% %d == 0, planes >= pixels*ps apart, offsets < 2^31", vec);
    return RDN_E_SHAPE;
  }
  const int taps = d->gather == RDN_G_CONV3 ? 9 : d->gather == RDN_G_S2 ? 4 : 1;
  if (taps * d->cin > d->kp) { rdn_set_error("rdn_conv_fwd: kp=%d < K=%d", d->kp, taps * d->cin); return RDN_E_SHAPE; }
  if (d->gather == RDN_G_S2 && (d->hin != 2 * d->h || d->win != 2 * d->w)) { rdn_set_error("rdn_conv_fwd: s2 grid mismatch"); return RDN_E_SHAPE; }
  if (d->gather != RDN_G_S2 && (d->hin != d->h || d->win != d->w)) { rdn_set_error("rdn_conv_fwd: grid mismatch"); return RDN_E_SHAPE; }
  if ((int64_t)d->n * d->h * d->w >= (1ll << 31)) { rdn_set_error("rdn_conv_fwd: too many pixels"); return RDN_E_SHAPE; }
  if ((d->flags & RDN_EPI_SCATTER2) && (d->cout * 4 != d->ncols || d->cout % vec || (d->flags & RDN_EPI_OUT_NCHW))) {
    rdn_set_error("rdn_conv_fwd: scatter needs ncols=4*cout, cout %% %d == 0, NHWC output", vec);
    return RDN_E_SHAPE;
  }
  if ((d->flags & RDN_EPI_OUT_NCHW) ? !d->out_nchw : !d->out) { rdn_set_error("rdn_conv_fwd: null output"); return RDN_E_ARG; }
  if ((d->flags & RDN_EPI_BIAS) && !d->bias) { rdn_set_error("rdn_conv_fwd: null bias"); return RDN_E_ARG; }
  if ((d->flags & RDN_EPI_PRELU) && !d->alpha) { rdn_set_error("rdn_conv_fwd: null alpha"); return RDN_E_ARG; }
  if ((d->flags & RDN_EPI_STORE_PRE) && !d->pre) { rdn_set_error("rdn_conv_fwd: null pre"); return RDN_E_ARG; }
  if ((d->flags & RDN_EPI_RESID) && !((d->flags & RDN_EPI_OUT_NCHW) ? (const void*)d->res_nchw : d->res)) {
    rdn_set_error("rdn_conv_fwd: null residual"); return RDN_E_ARG;
  }
  if (d->gout) {   // gate-out epilogue: an input gradient whose column tail is a layer's complete dY
    if (d->gather != RDN_G_CONV3 || !d->gout_pre || !d->gout_alpha || !d->gout_part ||
        (d->flags & ~(RDN_EPI_ACCUM | RDN_EPI_RESID)) || d->gout_c0 <= 0 || d->gout_c0 >= d->ncols ||
        d->gout_c0 % vec || d->ncols % vec || d->gout_ps % vec || d->gout_pre_ps % vec ||
        d->gout_ps < d->ncols - d->gout_c0 || d->gout_pre_ps < d->ncols - d->gout_c0 ||
        ((uintptr_t)d->gout & 15) || ((uintptr_t)d->gout_pre & 15)) {
      rdn_set_error("rdn_conv_fwd: gate-out needs a 3x3 input gradient (no bias/PReLU epilogue), 0 < gout_c0 < ncols, "
                    "16-byte units and rows");
      return RDN_E_ARG;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  if (d->gather == RDN_G_CONV3) return rdn_conv3_launch(d, st);  // LDS-halo kernel (conv3_halo.hip)
  if (d->gate) { rdn_set_error("rdn_conv_fwd: the PReLU gate is supported for RDN_G_CONV3 only"); return RDN_E_ARG; }
  if (RDN_PIX) {   // streaming register-weight GEMM of the bf16 2x2 / per-pixel shapes (conv_pix.hip)
    const int pix = rdn_conv_pix_launch(d, st);
    if (pix <= 0) return pix;
  }
  return d->dtype == RDN_BF16 ? launch_typed<bf16>(d, st) : launch_typed<float>(d, st);
}

// ---- split-K forward (round 6): the small-image convs of a batch-1 forward (config
// 1's RDUNet(64) on 1 x 3 x 64^2: the level-2/3 grids are 256 / 64 pixels, 4-64 blocks on
// 256 CUs; UNet/RDUNet_model.py:157-186).  The K walk is cut into slices that run as
// separate blocks, each storing its raw fp32 tile to ws[slice][m][ncols]; one reduce
// launch sums the slices in slice order (deterministic) and applies the conv epilogue
// (c3::finish_unit: bias, PReLU input, PReLU, residual, accumulate, NCHW output, with
// the depth-to-space scatter of the transposed conv).
namespace {

template <typename T>
__global__ __launch_bounds__(256) void conv_splitk_reduce_kernel(rdn_conv_desc d, const float* __restrict__ ws,
                                                                 int splits, FastDiv fd_w, FastDiv fd_hw) {
  constexpr int VEC = TypeInfo<T>::VEC;
  const int upr = (d.ncols + VEC - 1) / VEC;   // 16-B units per GEMM row
  const int64_t M = (int64_t)d.n * d.h * d.w;
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= M * upr) return;
  const int64_t m = u / upr;
  const int col = (int)(u - m * upr) * VEC;
  float v[VEC];
#pragma unroll
  for (int q = 0; q < VEC; ++q) v[q] = 0.f;
  const float* p = ws + m * d.ncols + col;
  const int64_t slice = M * d.ncols;
  int z = 0;
  if (col + VEC <= d.ncols) {
    // ZB slices' loads in flight at once, then summed in slice order (a dependent load per
    // slice ran 4.7 us at 2 slices, 12 us at 32, config 1's graph forward, r06)
    constexpr int ZB = 8;
    for (; z + ZB <= splits; z += ZB, p += ZB * slice) {
      f32x4 t[ZB][VEC / 4];
#pragma unroll
      for (int k = 0; k < ZB; ++k)
#pragma unroll
        for (int q = 0; q < VEC; q += 4) t[k][q / 4] = *(const f32x4*)(p + k * slice + q);
#pragma unroll
      for (int k = 0; k < ZB; ++k)
#pragma unroll
        for (int q = 0; q < VEC; q += 4) {
          v[q] += t[k][q / 4][0]; v[q + 1] += t[k][q / 4][1]; v[q + 2] += t[k][q / 4][2]; v[q + 3] += t[k][q / 4][3];
        }
    }
  }
#pragma unroll 4
  for (; z < splits; ++z, p += slice) {
    if (col + VEC <= d.ncols) {
#pragma unroll
      for (int q = 0; q < VEC; q += 4) {
        const f32x4 t4 = *(const f32x4*)(p + q);
        v[q] += t4[0]; v[q + 1] += t4[1]; v[q + 2] += t4[2]; v[q + 3] += t4[3];
      }
    } else {
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        if (col + q < d.ncols) v[q] += p[q];
    }
  }
  const int nimg = (int)fdiv((uint32_t)m, fd_hw);
  const int rem = (int)m - nimg * d.h * d.w;
  int y = (int)fdiv((uint32_t)rem, fd_w), x = rem - y * d.w, c = col;
  int64_t opix = m;
  if (d.flags & RDN_EPI_SCATTER2) {   // column tap * cout + c -> pixel (2y + dy, 2x + dx)
    const int tp = col / d.cout;
    c = col - tp * d.cout;
    y = 2 * y + (tp >> 1);
    x = 2 * x + (tp & 1);
    opix = ((int64_t)nimg * (2 * d.h) + y) * (2 * d.w) + x;
  }
  c3::finish_unit<T>(d, v, c, opix, y, x, nimg, c3::PF_NONE, u32x4{0u, 0u, 0u, 0u});
}

// the split rule's CU count (~2 blocks per CU as the target: 4 and 8 per CU measured the
// same on config 1's graph forward, 1.22 ms, r06)
int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        c <= 0)
      c = 256;
    cus = c;
  }
  return cus;
}

// slices of a 2x2 / per-pixel GEMM layer: as the 3x3 rule (conv3_halo.hip), over K stages
int gemm_splitk_slices(const rdn_conv_desc* d, int cus) {
  if (d->gather == RDN_G_CONV3 || d->gate || d->gout || d->ncols % 4) return 0;
  const int vec = d->dtype == RDN_BF16 ? 8 : 4, sk = 8 * vec;
  if ((d->flags & RDN_EPI_SCATTER2) && (d->cout % vec || d->cout * 4 != d->ncols)) return 0;
  const int taps = d->gather == RDN_G_S2 ? 4 : 1;
  const int nst = (taps * d->cin + sk - 1) / sk;
  const int bn = gemm_bn(d);
  const int64_t base = ((int64_t)d->n * d->h * d->w + 127) / 128 * ((d->ncols + bn - 1) / bn);
  if (nst < 2 || 2 * base > cus) return 0;
  int s = (int)((rdn_splitk_target(cus) + base - 1) / base);
  if (s > nst) s = nst;
  const int s_per = (nst + s - 1) / s;
  return (nst + s_per - 1) / s_per;
}

int splitk_slices(const rdn_conv_desc* d) {
  if (d->dtype != RDN_F32 && d->dtype != RDN_BF16) return 0;
  return d->gather == RDN_G_CONV3 ? rdn_conv3_splitk_slices(d, device_cus()) : gemm_splitk_slices(d, device_cus());
}

}  // namespace

extern "C" int32_t rdn_conv_fwd_splits(const rdn_conv_desc* d) {
  if (!d) { rdn_set_error("rdn_conv_fwd_splits: null"); return RDN_E_ARG; }
  return splitk_slices(d);
}

extern "C" int64_t rdn_conv_fwd_splitk_workspace_size(const rdn_conv_desc* d, int32_t splits) {
  if (!d || splits <= 0) return RDN_E_ARG;
  return (int64_t)splits * d->n * d->h * d->w * d->ncols * (int64_t)sizeof(float);
}

extern "C" int rdn_conv_fwd_splitk(const rdn_conv_desc* d, int32_t splits, float* ws, void* stream) {
  if (!d || !ws || ((uintptr_t)ws & 15)) { rdn_set_error("rdn_conv_fwd_splitk: null / unaligned workspace"); return RDN_E_ARG; }
  if (splits <= 0) return rdn_conv_fwd(d, stream);
  if (splits != splitk_slices(d)) {
    rdn_set_error("rdn_conv_fwd_splitk: splits %d != rdn_conv_fwd_splits %d for this descriptor", splits, splitk_slices(d));
    return RDN_E_ARG;
  }
  if (!d->x || !d->wp || d->cin % 8 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15)) {
    rdn_set_error("rdn_conv_fwd_splitk: null / unaligned operand, cin %% 8");
    return RDN_E_ARG;
  }
  const int taps = d->gather == RDN_G_CONV3 ? 9 : d->gather == RDN_G_S2 ? 4 : 1;
  if (d->gather == RDN_G_CONV3 ? d->kp < rdn_conv3_packed_k(d->cin, d->dtype) : taps * d->cin > d->kp) {
    rdn_set_error("rdn_conv_fwd_splitk: kp=%d too small", d->kp);
    return RDN_E_SHAPE;
  }
  if (d->gather == RDN_G_S2 ? (d->hin != 2 * d->h || d->win != 2 * d->w) : (d->hin != d->h || d->win != d->w)) {
    rdn_set_error("rdn_conv_fwd_splitk: grid mismatch");
    return RDN_E_SHAPE;
  }
  if ((d->flags & RDN_EPI_OUT_NCHW) ? !d->out_nchw : !d->out) { rdn_set_error("rdn_conv_fwd_splitk: null output"); return RDN_E_ARG; }
  if (((d->flags & RDN_EPI_BIAS) && !d->bias) || ((d->flags & RDN_EPI_PRELU) && !d->alpha) ||
      ((d->flags & RDN_EPI_STORE_PRE) && !d->pre) ||
      ((d->flags & RDN_EPI_RESID) && !((d->flags & RDN_EPI_OUT_NCHW) ? (const void*)d->res_nchw : d->res))) {
    rdn_set_error("rdn_conv_fwd_splitk: epilogue operand missing");
    return RDN_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if (d->gather == RDN_G_CONV3) rc = rdn_conv3_splitk_launch(d, splits, ws, st);
  else rc = d->dtype == RDN_BF16 ? launch_typed<bf16>(d, st, splits, ws) : launch_typed<float>(d, st, splits, ws);
  if (rc) return rc;
  const int vec = d->dtype == RDN_BF16 ? 8 : 4;
  const int64_t units = (int64_t)d->n * d->h * d->w * ((d->ncols + vec - 1) / vec);
  const unsigned blocks = (unsigned)((units + 255) / 256);
  FastDiv fw = make_fastdiv((uint32_t)d->w), fhw = make_fastdiv((uint32_t)(d->h * d->w));
  RDN_PROBE("conv_splitk_reduce_kernel<%s>", d->dtype == RDN_BF16 ? "bf16" : "f32");
  if (d->dtype == RDN_BF16) conv_splitk_reduce_kernel<bf16><<<blocks, 256, 0, st>>>(*d, ws, splits, fw, fhw);
  else conv_splitk_reduce_kernel<float><<<blocks, 256, 0, st>>>(*d, ws, splits, fw, fhw);
  return rdn_check_launch("rdn_conv_fwd_splitk(reduce)");
}
