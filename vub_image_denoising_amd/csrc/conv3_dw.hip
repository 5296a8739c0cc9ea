// Fused input gradient + weight gradient of the narrow level-0 3x3 convolutions
// (gfx950): one pass over a layer's gated output gradient produces BOTH
//
//   dX[p][ci]  (+)=  sum_{tap, co} W[co][ci][tap] * dYpre[p - tap + 1][co]      (dgrad)
//   ws[split][co][tap*ndim + ci] = sum_p dYpre[p][co] * X[p + tap - 1][ci]      (wgrad)
//   part[split][0|1][co]         = sum_p (pre <= 0 ? pre*dY : 0) | dYpre      (dalpha, dbias)
//
// with dYpre = dY * (pre > 0 ? 1 : alpha) computed in the loader (aten
// _prelu_kernel_backward + convolution_backward of Unet_model.py:72-89's
// DenoisingBlock convs, level 0: 16-32 output channels, 32-80 input channels).
//
// Why fused: as two kernels (conv3_ws gated dgrad on the compute stream, the rows
// weight gradient on the side stream) each re-reads dY and the saved PReLU input,
// and the two co-run on the same CUs at ~0.27 of HBM each (trace r02_v6: the
// 80->32 pair costs 280 us of wall per layer).  Here the block stages, per 8 x 16
// tile, the gated dY halo [(8+2) x (16+2)][CK] and the input halo X [(8+2) x
// (16+2)][BN] in LDS ONCE and runs both GEMMs from them:
//
//   dgrad: M = 128 tile pixels (wave w = tile row w), N = BN input channels,
//          K = 9 taps x CK, A = dY halo (ds_read_b128), B = resident weight panel;
//   wgrad: M = CK output channels, N = 9 x BN (tap, ci) columns (wave w owns
//          n-tiles w, w+8, ...), K = the 128 tile pixels, A = the dY halo's
//          interior and B = the X halo shifted per tap, both k-major fragments by
//          ds_read_b64_tr_b16 (same k order as wgrad3_rows: lane group g takes
//          pixels 4g..4g+3 then 16+4g..16+4g+3 of a 32-pixel k-step).
//
// Persistent grid, one 8-wave block per CU, XCD-local tile ranges (as conv3_ws);
// the weight-gradient accumulators stay in registers over the block's tiles and
// the block writes ONE split-K slab at the end (split = block), summed with the
// dalpha/dbias partials by rdn_wgrad_reduce in fixed order (deterministic).  The
// next tile's halos (and the epilogue's residual / accumulate operands) are in
// flight in registers while the current tile computes.
#include "conv3_tile.h"

#include <stdlib.h>

namespace {

using c3::BM;
using c3::HW_;
using c3::TH;
using c3::TW;

constexpr int NT = 512;   // 8 waves
constexpr int LDS_MAX = 160 * 1024;

template <int BN, int CK>
struct DwCfg {
  static constexpr int KC = (9 * CK + 63) / 64 * 64;   // packed dgrad K (rdn_pack_weights, conv3_ws)
  static constexpr int NSTEP = KC / 32;
  static constexpr int WROW = KC * 2 + 32;              // = 32 mod 128: conflict-free B reads
  static constexpr int W_BYTES = BN * WROW;
  static constexpr int DROW = c3::HaloRow<CK * 2>::V;   // dY halo row stride (b128 and tr16 conflict-free)
  static constexpr int XROW = c3::HaloRow<BN * 2>::V;   // X halo row stride
  static constexpr int D_BYTES = (HW_ * DROW + 15) / 16 * 16;
  static constexpr int X_BYTES = (HW_ * XROW + 15) / 16 * 16;
  static constexpr int CROWF = BN + 4;                  // epilogue fp32 row (floats)
  static constexpr int CT_BYTES = BM * CROWF * 4;
  static constexpr int RED_BYTES = 2 * NT * 8 * 4;      // dalpha/dbias partial reduction (aliases)
  static constexpr int AL_BYTES = (CK * 4 + 15) / 16 * 16;   // gate slopes
  static constexpr int LDS = W_BYTES + D_BYTES + X_BYTES + CT_BYTES + AL_BYTES;
  static constexpr bool FITS = LDS <= LDS_MAX && D_BYTES + X_BYTES + CT_BYTES >= RED_BYTES;
};

template <int BN, int CK>
__global__ __launch_bounds__(NT, 1) void conv3_dw_kernel(rdn_conv_desc d, rdn_wgrad_desc wg, int tiles_x, int tiles_y,
                                                         int ntiles, int dbg) {
  using Cfg = DwCfg<BN, CK>;
  constexpr int VEC = 8;
  constexpr int KC = Cfg::KC, NSTEP = Cfg::NSTEP, WROW = Cfg::WROW, DROW = Cfg::DROW, XROW = Cfg::XROW;
  constexpr int CROWF = Cfg::CROWF;
  constexpr int NTL = BN / 16;                          // dgrad n-tiles
  constexpr int DU = CK / VEC, XU = BN / VEC;           // 16-B units per halo pixel
  constexpr int D_UNITS = HW_ * DU, X_UNITS = HW_ * XU;
  constexpr int D_IT = (D_UNITS + NT - 1) / NT, X_IT = (X_UNITS + NT - 1) / NT;
  constexpr int MTW = CK / 16;                          // wgrad m-tiles
  constexpr int NT_ALL = 9 * BN / 16;                   // wgrad n-tiles
  constexpr int NTW = (NT_ALL + 7) / 8;                 // per wave (n-tile = wave + 8 j)
  constexpr int UPR = BN / VEC, EU = BM * UPR, E_IT = (EU + NT - 1) / NT;
  constexpr bool KALIGN = CK % 32 == 0;                 // a dgrad k-step never straddles a tap
  constexpr int RS = (TW + 2);                          // halo pixels per halo row
  static_assert(NT % DU == 0, "fixed dY channel group per thread");
  static_assert(BN % 16 == 0 && CK % 16 == 0, "16-wide MFMA tiles");
  static_assert(Cfg::FITS, "LDS");

  __shared__ __attribute__((aligned(16))) unsigned char lds[Cfg::LDS];
  unsigned char* const wl = lds;
  unsigned char* const dyh = lds + Cfg::W_BYTES;
  unsigned char* const xh = dyh + Cfg::D_BYTES;
  float* const Ct = (float*)(xh + Cfg::X_BYTES);
  float* const alds = (float*)(xh + Cfg::X_BYTES + Cfg::CT_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int H = d.h, W = d.w;
  const int flags = d.flags;

  // this block's tiles: XCD share, strided by the XCD's block count (conv3_ws)
  const int per = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7;
  const int t_hi = (int)((int64_t)ntiles * (xcd + 1) / 8);
  int t = (int)((int64_t)ntiles * xcd / 8) + (blockIdx.x >> 3);

  const bf16* __restrict__ DY = (const bf16*)d.x;
  const bf16* __restrict__ PR = (const bf16*)d.gate;
  const bf16* __restrict__ XS = (const bf16*)wg.b;

  // ---- resident dgrad weight panel: BN rows x KC
  {
    const bf16* __restrict__ WP = (const bf16*)d.wp;
    constexpr int UPRW = KC / VEC;
    for (int u = tid; u < BN * UPRW; u += NT) {
      const int n = u / UPRW, k8 = u - n * UPRW;
      *(u32x4*)(wl + n * WROW + k8 * 16) = *(const u32x4*)(WP + (int64_t)n * d.kp + k8 * VEC);
    }
    for (int c = tid; c < CK; c += NT) alds[c] = d.gate_alpha[c];
  }

  // ---- loader geometry (tile-invariant): dY + gate pixel-major with a fixed channel
  // group per thread; X plane-major when channel-blocked (a load instruction walks
  // consecutive pixels of one plane)
  const int dcu = tid % DU;
  int drel[D_IT], grel[D_IT], dhp[D_IT];
  unsigned dint = 0;   // bit it: unit `it` is a tile-interior pixel (counted in the partials)
#pragma unroll
  for (int it = 0; it < D_IT; ++it) {
    const int u = tid + it * NT;
    const int hp = u < D_UNITS ? u / DU : HW_ - 1;
    const int hy = hp / RS, hx = hp - hy * RS;
    dhp[it] = hp;
    drel[it] = (hy * W + hx) * (int)d.x_ps + rdn_coff32(d.x_c0 + dcu * VEC, (int)d.x_ps, (int)d.x_pl);
    grel[it] = (hy * W + hx) * (int)d.gate_ps + rdn_coff32(dcu * VEC, (int)d.gate_ps, (int)d.gate_pl);
    if (u < D_UNITS && hy >= 1 && hy <= TH && hx >= 1 && hx <= TW) dint |= 1u << it;
  }
  const int xupp = (wg.b_pl && wg.b_c0 % wg.b_ps == 0 && XU % (wg.b_ps / VEC) == 0) ? (int)(wg.b_ps / VEC) : XU;
  int xrel[X_IT], xlds[X_IT];
#pragma unroll
  for (int it = 0; it < X_IT; ++it) {
    const int u = tid + it * NT;
    const int pln = u / (HW_ * xupp), rem = u - pln * (HW_ * xupp);
    const int hp = u < X_UNITS ? rem / xupp : HW_ - 1, cu = u < X_UNITS ? pln * xupp + rem % xupp : 0;
    const int hy = hp / RS, hx = hp - hy * RS;
    xrel[it] = (hy * W + hx) * (int)wg.b_ps + rdn_coff32(wg.b_c0 + cu * VEC, (int)wg.b_ps, (int)wg.b_pl);
    xlds[it] = hp * XROW + cu * 16;
  }
  float sa[VEC], sb[VEC];
#pragma unroll
  for (int q = 0; q < VEC; ++q) {
    sa[q] = 0.f;
    sb[q] = 0.f;
  }

  // ---- epilogue units (dX): pixel offset in the tile + channel
  int erel[E_IT], ecol[E_IT];
#pragma unroll
  for (int it = 0; it < E_IT; ++it) {
    const int u = tid + it * NT;
    const int px = u / UPR;
    erel[it] = (px / TW) * W + px % TW;
    ecol[it] = (u - px * UPR) * VEC;
  }
  const bool has_res = flags & RDN_EPI_RESID, has_acc = flags & RDN_EPI_ACCUM;

  auto origin = [&](int tt, int& oy, int& ox, int& on) {
    const int tx = tt % tiles_x;
    tt /= tiles_x;
    oy = (tt % tiles_y) * TH;
    ox = tx * TW;
    on = tt / tiles_y;
  };
  auto load_halos = [&](int oy, int ox, int on, u32x4 (&dr)[D_IT], u32x4 (&gr)[D_IT], u32x4 (&xr)[X_IT]) {
    const int64_t hpix0 = ((int64_t)on * H + (oy - 1)) * W + (ox - 1);
    const bf16* const db = DY + hpix0 * d.x_ps;
    const bf16* const gb = PR + hpix0 * d.gate_ps;
    const bf16* const xb = XS + hpix0 * wg.b_ps;
    const bool interior = oy >= 1 && oy + TH + 1 <= H && ox >= 1 && ox + TW + 1 <= W;
#pragma unroll
    for (int it = 0; it < D_IT; ++it) {
      bool ok = (it + 1 < D_IT) || tid + it * NT < D_UNITS;
      if (!interior) {
        const int hy = dhp[it] / RS, hx = dhp[it] - (dhp[it] / RS) * RS;
        ok = ok && (unsigned)(oy - 1 + hy) < (unsigned)H && (unsigned)(ox - 1 + hx) < (unsigned)W;
      }
      u32x4 v = {0u, 0u, 0u, 0u}, gv = {0u, 0u, 0u, 0u};
      if (ok) {
        v = *(const u32x4*)(db + drel[it]);
        gv = *(const u32x4*)(gb + grel[it]);
      }
      dr[it] = v;
      gr[it] = gv;
    }
#pragma unroll
    for (int it = 0; it < X_IT; ++it) {
      bool ok = (it + 1 < X_IT) || tid + it * NT < X_UNITS;
      if (!interior) {
        const int hp = xlds[it] / XROW;
        const int hy = hp / RS, hx = hp - hy * RS;
        ok = ok && (unsigned)(oy - 1 + hy) < (unsigned)H && (unsigned)(ox - 1 + hx) < (unsigned)W;
      }
      u32x4 v = {0u, 0u, 0u, 0u};
      if (ok) v = *(const u32x4*)(xb + xrel[it]);
      xr[it] = v;
    }
  };
  // registers -> LDS; the PReLU-backward gate and the dalpha/dbias partials of the
  // tile-interior pixels (each image pixel is interior to exactly one tile)
  auto store_halos = [&](const u32x4 (&dr)[D_IT], const u32x4 (&gr)[D_IT], const u32x4 (&xr)[X_IT]) {
#pragma unroll
    for (int it = 0; it < D_IT; ++it) {
      if (it + 1 == D_IT && tid + it * NT >= D_UNITS) continue;
      float dy[VEC], pr[VEC];
      Unit16<bf16>::unpack(dr[it], dy);
      Unit16<bf16>::unpack(gr[it], pr);
      const bool in = (dint >> it) & 1u;
      const f32x4 a0 = *(const f32x4*)(alds + dcu * VEC), a1 = *(const f32x4*)(alds + dcu * VEC + 4);
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const bool pos = pr[q] > 0.f;
        if (in && !pos) sa[q] += pr[q] * dy[q];
        dy[q] = pos ? dy[q] : (q < 4 ? a0[q] : a1[q - 4]) * dy[q];
        if (in) sb[q] += dy[q];
      }
      *(u32x4*)(dyh + dhp[it] * DROW + dcu * 16) = Unit16<bf16>::pack(dy);
    }
#pragma unroll
    for (int it = 0; it < X_IT; ++it) {
      if (it + 1 == X_IT && tid + it * NT >= X_UNITS) continue;
      *(u32x4*)(xh + xlds[it]) = xr[it];
    }
  };
  // epilogue operand (residual, else the accumulated output) of a tile, one tile ahead
  auto load_epi = [&](int oy, int ox, int on, u32x4 (&eo)[E_IT]) {
    if (!has_res && !has_acc) return;
    const int64_t opix0 = ((int64_t)on * H + oy) * W + ox;
#pragma unroll
    for (int it = 0; it < E_IT; ++it) {
      if (it + 1 == E_IT && tid + it * NT >= EU) continue;
      const int c = ecol[it];
      const int64_t opix = opix0 + erel[it];
      if (has_res) {
        if (c < d.res_climit)
          eo[it] = *(const u32x4*)((const bf16*)d.res + opix * d.res_ps +
                                   rdn_coff32(d.res_c0 + c, (int)d.res_ps, (int)d.res_pl));
      } else {
        eo[it] = *(const u32x4*)((const bf16*)d.out + opix * d.out_ps +
                                 rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl));
      }
    }
  };

  // ---- fragment addressing (per lane, tile-invariant)
  // dgrad A: pixel r of tile row `wave`; k-step j covers k = 32 j + 8 g
  const int a_lane = (wave * RS + r) * DROW;
  int offA[KALIGN ? 1 : NSTEP];
  if constexpr (!KALIGN) {
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      const int k = 32 * j + 8 * g;
      int tap = k / CK;
      const int ci = k - tap * CK;
      tap = tap < 9 ? tap : 8;   // padded k: zero weights, finite operand
      offA[j] = a_lane + ((tap / 3) * RS + tap % 3) * DROW + ci * 2;
    }
  }
  const unsigned char* const pda = dyh + (KALIGN ? a_lane + g * 16 : 0);
  const unsigned char* const pdb = wl + r * WROW + g * 16;
  // wgrad: lane (g, q = r>>2, pp = r&3) supplies pixels {4g+q, 16+4g+q} of each
  // 32-pixel k-step (tile rows 2ks, 2ks+1) and channels / columns 4pp..4pp+3
  const int q4 = r >> 2, pp = r & 3;
  const unsigned char* const pwa = dyh + (RS + 4 * g + q4 + 1) * DROW + 4 * pp * 2;   // interior (0, 4g+q)
  const unsigned char* const pwb = xh + (4 * g + q4) * XROW;
  int boff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + 8 * j;
    const int c = nt < NT_ALL ? nt * 16 + 4 * pp : 0;
    const int tp = c / BN, ci = c - (c / BN) * BN;
    boff[j] = ((tp / 3) * RS + tp % 3) * XROW + ci * 2;
  }

  f32x4 accW[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) accW[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute_tile = [&]() {
    // input gradient of the tile: 16 pixels x BN columns per wave
    f32x4 accD[NTL];
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) accD[jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (!(dbg & 1))
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      int ao;
      if constexpr (KALIGN) {
        const int k0 = 32 * j;
        int tap = k0 / CK;
        const int ci = k0 - tap * CK;
        tap = tap < 9 ? tap : 8;
        ao = ((tap / 3) * RS + tap % 3) * DROW + ci * 2;
      } else {
        ao = offA[j];
      }
      const u32x4 af = *(const u32x4*)(pda + ao);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        const u32x4 bfr = *(const u32x4*)(pdb + jn * 16 * WROW + j * 64);
        accD[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af),
                                                           __builtin_bit_cast(bf16x8, bfr), accD[jn], 0, 0, 0);
      }
    }
    // weight gradient: K = the tile's 128 pixels, 4 k-steps
    if (!(dbg & 2))
#pragma unroll
    for (int ks = 0; ks < TH / 2; ++ks) {
      bf16x8 af[MTW];
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, pwa + (2 * ks) * RS * DROW + i * 32));
        const i16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, pwa + (2 * ks + 1) * RS * DROW + i * 32));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        if (wave + 8 * j >= NT_ALL) continue;   // wave-uniform
        const unsigned char* b = pwb + boff[j] + (2 * ks) * RS * XROW;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b + RS * XROW));
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int i = 0; i < MTW; ++i) accW[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, accW[i][j], 0, 0, 0);
      }
    }
    // fp32 dX tile to LDS: D[m = pixel][n = column], lane rows g*4+e, column r
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn)
#pragma unroll
      for (int e = 0; e < 4; ++e) Ct[(wave * 16 + g * 4 + e) * CROWF + jn * 16 + r] = accD[jn][e];
  };
  auto epilogue = [&](int oy, int ox, int on, const u32x4 (&eo)[E_IT]) {
    const int64_t opix0 = ((int64_t)on * H + oy) * W + ox;
#pragma unroll
    for (int it = 0; it < E_IT; ++it) {
      const int u = tid + it * NT;
      if (it + 1 == E_IT && u >= EU) continue;
      const int c = ecol[it];
      float v[VEC];
      const float* src = Ct + (u / UPR) * CROWF + c;
#pragma unroll
      for (int q = 0; q < VEC; q += 4) {
        const f32x4 t4 = *(const f32x4*)(src + q);
        v[q] = t4[0]; v[q + 1] = t4[1]; v[q + 2] = t4[2]; v[q + 3] = t4[3];
      }
      const int64_t opix = opix0 + erel[it];
      if ((has_res && c < d.res_climit) || has_acc) {
        float rv[VEC];
        Unit16<bf16>::unpack(eo[it], rv);
#pragma unroll
        for (int q = 0; q < VEC; ++q) v[q] += rv[q];
      }
      *(u32x4*)((bf16*)d.out + opix * d.out_ps + rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl)) =
          Unit16<bf16>::pack(v);
    }
  };

  // ---- the tile loop: LDS holds tile t; the next tile's loads are in flight
  u32x4 dA[D_IT], gA[D_IT], xA[X_IT], eC[E_IT], eN[E_IT];
  int y0 = 0, x0 = 0, nimg = 0;
  if (t < t_hi) {
    origin(t, y0, x0, nimg);
    load_halos(y0, x0, nimg, dA, gA, xA);
    load_epi(y0, x0, nimg, eC);
    store_halos(dA, gA, xA);
  }
  __syncthreads();   // weights + first halos
  while (t < t_hi) {
    const int t1 = t + per;
    int y1 = 0, x1 = 0, n1 = 0;
    if (t1 < t_hi) {
      origin(t1, y1, x1, n1);
      load_epi(y1, x1, n1, eN);
      load_halos(y1, x1, n1, dA, gA, xA);
    }
    compute_tile();
    __syncthreads();   // halos consumed, dX tile complete in Ct
    if (t1 < t_hi) store_halos(dA, gA, xA);
    if (!(dbg & 4)) epilogue(y0, x0, nimg, eC);
    __syncthreads();   // next halos visible, Ct consumed
#pragma unroll
    for (int it = 0; it < E_IT; ++it) eC[it] = eN[it];
    t = t1; y0 = y1; x0 = x1; nimg = n1;
  }

  // ---- this block's split: weight-gradient slab (zero for a block without tiles)
  const int ncol_all = 9 * wg.ndim;
  float* __restrict__ ws = wg.ws + (int64_t)blockIdx.x * wg.mdim * ncol_all;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + 8 * j;
    if (nt >= NT_ALL) continue;
    const int c = nt * 16 + r;
    const int tp = c / BN, ci = c - tp * BN;
    const int col = tp * wg.ndim + ci;
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = i * 16 + g * 4 + e;
        if (m < wg.mdim) ws[(int64_t)m * ncol_all + col] = accW[i][j][e];
      }
  }
  // ---- dalpha / dbias partials of this split, fixed order
  if (wg.part) {
    float* red = (float*)(lds + Cfg::W_BYTES);   // the loop ended with a barrier
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      red[tid * VEC + k] = sa[k];
      red[NT * VEC + tid * VEC + k] = sb[k];
    }
    __syncthreads();
    if (tid < CK) {
      const int cg = tid / VEC, k = tid % VEC;
      float a = 0.f, b = 0.f;
      for (int rr = 0; rr < NT / DU; ++rr) {
        a += red[(rr * DU + cg) * VEC + k];
        b += red[NT * VEC + (rr * DU + cg) * VEC + k];
      }
      if (tid < wg.mdim) {
        wg.part[((int64_t)blockIdx.x * 2 + 0) * wg.mdim + tid] = a;
        wg.part[((int64_t)blockIdx.x * 2 + 1) * wg.mdim + tid] = b;
      }
    }
  }
}

bool dw_enabled() {
  static const bool on = [] {
    const char* e = getenv("RDN_DW");
    return !(e && e[0] == '0');
  }();
  return on;
}

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8) n = 256;
    cus = n;
  }
  return cus;
}

// blocks of the persistent grid = the weight-gradient split count: one per CU (a
// multiple of 8: the XCD tile ranges), at most the tiles of an XCD's share
int dw_grid(int ntiles) {
  const int per_xcd = (ntiles + 7) / 8;
  int slots = device_cus() / 8;
  if (slots > per_xcd) slots = per_xcd;
  if (slots < 1) slots = 1;
  return 8 * slots;
}

// the pair this kernel serves (else 1 = run the separate dgrad / wgrad launches)
bool dw_serves(const rdn_conv_desc* d, const rdn_wgrad_desc* wg) {
  if (!dw_enabled() || !d || !wg) return false;
  if (d->dtype != RDN_BF16 || wg->dtype != RDN_BF16 || d->gather != RDN_G_CONV3 || wg->gather != RDN_G_CONV3) return false;
  if (!d->gate || !wg->a_gate || !d->gate_alpha || d->bn || d->bm) return false;
  if (d->flags & ~(RDN_EPI_RESID | RDN_EPI_ACCUM)) return false;
  if (d->h % TH || d->w % TW || d->n != wg->n || d->h != wg->h || d->w != wg->w) return false;
  if (d->cin != 16 && d->cin != 32) return false;
  if (d->ncols != d->cout || d->ncols % 16 || d->ncols < 32 || d->ncols > 80 || wg->ndim != d->ncols) return false;
  if (wg->mdim > d->cin || wg->mdim <= 0 || wg->b_c0 % 8 || wg->b_ps % 8 || ((uintptr_t)wg->b & 15)) return false;
  // the same gated operand on both sides
  if (wg->a != d->x || wg->a_ps != d->x_ps || wg->a_c0 != d->x_c0 || wg->a_pl != d->x_pl || wg->a_gate != d->gate ||
      wg->a_gate_ps != d->gate_ps || wg->a_gate_pl != d->gate_pl || wg->a_gate_alpha != d->gate_alpha)
    return false;
  if (d->x_ps % 8 || d->x_c0 % 8 || d->gate_ps % 8 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->gate & 15)) return false;
  if (((uintptr_t)d->wp & 15) || d->kp % 8 || d->kp < (9 * d->cin + 63) / 64 * 64) return false;
  if (d->out_ps % 8 || d->out_c0 % 8 || ((uintptr_t)d->out & 15)) return false;
  if ((d->flags & RDN_EPI_RESID) && (d->res_climit % 8 || d->res_ps % 8 || d->res_c0 % 8 || ((uintptr_t)d->res & 15)))
    return false;
  // 32-bit per-thread offsets
  const int64_t span = (int64_t)(TH + 2) * d->w;
  if (span * d->x_ps >= (1ll << 30) || span * wg->b_ps >= (1ll << 30) || span * d->gate_ps >= (1ll << 30) ||
      (int64_t)TH * d->w * d->out_ps >= (1ll << 30) || (int64_t)TH * d->w * d->res_ps >= (1ll << 30))
    return false;
  if ((d->x_pl && rdn_coff(d->x_c0 + d->cin - 1, d->x_ps, d->x_pl) >= (1ll << 31)) ||
      (wg->b_pl && rdn_coff(wg->b_c0 + wg->ndim - 1, wg->b_ps, wg->b_pl) >= (1ll << 31)) ||
      (d->out_pl && rdn_coff(d->out_c0 + d->ncols - 1, d->out_ps, d->out_pl) >= (1ll << 31)) ||
      (d->res_pl && rdn_coff(d->res_c0 + d->res_climit - 1, d->res_ps, d->res_pl) >= (1ll << 31)) ||
      (d->gate_pl && rdn_coff(d->cin - 1, d->gate_ps, d->gate_pl) >= (1ll << 31)))
    return false;
  const int64_t nt = (int64_t)d->n * (d->h / TH) * (d->w / TW);
  return nt < (1ll << 31);
}

template <int BN, int CK>
int launch_dw(const rdn_conv_desc* d, const rdn_wgrad_desc* wg, hipStream_t st) {
  if constexpr (!DwCfg<BN, CK>::FITS) {
    return 1;
  } else {
    const int tiles_x = d->w / TW, tiles_y = d->h / TH;
    const int ntiles = d->n * tiles_x * tiles_y;
    const int grid = dw_grid(ntiles);
    RDN_PROBE("conv3_dw_kernel<bf16,%d,%d>", BN, CK);
    if (wg->splits != grid) {
      rdn_set_error("rdn_conv_dgrad_wgrad: wgrad splits %d != %d (rdn_conv_dgrad_wgrad_splits)", wg->splits, grid);
      return RDN_E_ARG;
    }
    if (!wg->ws) { rdn_set_error("rdn_conv_dgrad_wgrad: null workspace"); return RDN_E_ARG; }
    static const int dbg = [] {   // RDN_DW_DBG (diagnosis only, wrong results): 1 no dgrad MFMA,
      const char* e = getenv("RDN_DW_DBG");   // 2 no wgrad MFMA, 4 no dX stores
      return e ? atoi(e) : 0;
    }();
    hipLaunchKernelGGL((conv3_dw_kernel<BN, CK>), dim3((unsigned)grid), dim3(NT), 0, st, *d, *wg, tiles_x, tiles_y,
                       ntiles, dbg);
    return rdn_check_launch("rdn_conv_dgrad_wgrad");
  }
}

template <int CK>
int dw_bn(const rdn_conv_desc* d, const rdn_wgrad_desc* wg, hipStream_t st) {
  switch (d->ncols) {
    case 32: return launch_dw<32, CK>(d, wg, st);
    case 48: return launch_dw<48, CK>(d, wg, st);
    case 64: return launch_dw<64, CK>(d, wg, st);
    case 80: return launch_dw<80, CK>(d, wg, st);
  }
  return 1;
}

int dw_dispatch(const rdn_conv_desc* d, const rdn_wgrad_desc* wg, hipStream_t st) {
  if (!dw_serves(d, wg)) return 1;
  return d->cin == 32 ? dw_bn<32>(d, wg, st) : dw_bn<16>(d, wg, st);
}

}  // namespace

// Fused gated input gradient + weight gradient of one 3x3 conv (the level-0 layers).
// 0 = launched, 1 = this pair is not served (run rdn_conv_fwd(dgrad) and
// rdn_conv_wgrad(wgrad) instead), < 0 = error.
extern "C" int rdn_conv_dgrad_wgrad(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad, void* stream) {
  if (!dgrad || !wgrad) { rdn_set_error("rdn_conv_dgrad_wgrad: null descriptor"); return RDN_E_ARG; }
  return dw_dispatch(dgrad, wgrad, (hipStream_t)stream);
}

// split count (= persistent grid) the fused kernel writes for this pair, 0 if not served
extern "C" int rdn_conv_dgrad_wgrad_splits(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad) {
  if (!dw_serves(dgrad, wgrad)) return 0;
  char buf[8];
  rdn_probe_buf = buf;
  rdn_probe_len = (int)sizeof(buf);
  const int rc = dw_dispatch(dgrad, wgrad, nullptr);   // instantiation exists for this shape?
  rdn_probe_buf = nullptr;
  if (rc != 0) return 0;
  return dw_grid(dgrad->n * (dgrad->h / TH) * (dgrad->w / TW));
}

extern "C" int rdn_conv_dgrad_wgrad_kernel_name(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad, char* buf,
                                                int32_t len) {
  if (!buf || len < 1) { rdn_set_error("rdn_conv_dgrad_wgrad_kernel_name: no buffer"); return RDN_E_ARG; }
  buf[0] = 0;
  if (!dgrad || !wgrad || !dw_serves(dgrad, wgrad)) return 1;
  rdn_probe_buf = buf;
  rdn_probe_len = len;
  const int rc = dw_dispatch(dgrad, wgrad, nullptr);
  rdn_probe_buf = nullptr;
  return rc;
}
