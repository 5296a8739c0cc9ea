// Weight-stationary, persistent 3x3 / pad 1 convolution for the narrow layers
// (bf16, input channels <= 96 in ONE chunk, output columns <= 96): level 0 of
// the network at 256x256 (Unet_model.py:48-49,60-61,72-75 forward, and the
// input gradients of the same convs).  These layers move 100-300 MB per launch
// and carry little arithmetic, so the limit is HBM latency hiding, not MFMA.
//
// conv3_halo.hip streams the weights through LDS one 128-B K stage at a time
// (a barrier and an L2 round trip per stage: 5-15 dependent round trips per
// 8x16 tile at these shapes).  Here the block's whole packed weight panel
// (BN x KC bf16, <= ~64 KB) is loaded into LDS ONCE, and the block then loops
// over output tiles (persistent grid of 1-2 blocks per CU):
//
//   halo(t) in LDS --> 9 taps x MFMA  (no barriers inside the K loop)
//   halo(t+1) global loads in flight in registers meanwhile
//   epilogue of t (fp32 tile staged in LDS, 16-B NHWC stores), then halo(t+1) -> LDS
//
// Work split (XCD-aware): block b runs on XCD b % 8 (round-robin dispatch);
// XCD x owns tiles [x*T/8, (x+1)*T/8), its blocks take consecutive tiles of
// that range in lock step, so the tiles in flight on one XCD are adjacent and
// their overlapping halos are read through the same L2.
//
// Same packed layout and epilogue flags as conv3_halo (P[n][tap*CK + ci], KC =
// roundup(9*CK, 64)); GATE = PReLU backward fused into the halo loader.
#include "conv3_tile.h"

#include <stdlib.h>

namespace {

constexpr int NT = 256;
using c3::BM;
using c3::HW_;
using c3::TH;
using c3::TW;

constexpr int LDS_2BLK = 80 * 1024;     // two resident blocks per CU below this
// accumulator epilogue (<= 64 columns) in 16-byte units (pixel-row pairs swapped between
// lane rows); fragments read k-step by k-step (reading k-steps ahead measured no gain, r05)
constexpr int LDS_MAX = 160 * 1024;

template <int BN, int CK>
struct WsCfg {
  static constexpr int SK = 64;                          // k per 128-B stage
  static constexpr int KC = (9 * CK + SK - 1) / SK * SK;
  static constexpr int NSTG = KC / SK;
  static constexpr int WROW = KC * 2 + 32;               // bytes, = 32 mod 128: conflict-free B reads
  static constexpr int W_BYTES = BN * WROW;
  static constexpr int HROW = c3::HaloRow<CK * 2>::V;
  static constexpr int HALO_BYTES = HW_ * HROW;
  static constexpr int NTL = BN / 16;
  static constexpr int epi_bytes(int ntp) { return BM * (ntp * 64 + 16); }
  static constexpr int mx(int a, int b) { return a > b ? a : b; }
  // epilogue column passes: as wide as fits beside the weights in two-block LDS
  static constexpr int pick_ntp() {
    for (int t = NTL; t >= 1; --t)
      if (W_BYTES + mx(HALO_BYTES, epi_bytes(t)) <= LDS_2BLK) return t;
    for (int t = NTL; t > 1; --t)   // one block per CU anyway: widest pass that fits
      if (W_BYTES + mx(HALO_BYTES, epi_bytes(t)) <= LDS_MAX) return t;
    return 1;
  }
  static constexpr int NTP = pick_ntp();
  static constexpr int NPASS = (NTL + NTP - 1) / NTP;
  static constexpr int R2 = mx(HALO_BYTES, epi_bytes(NTP));
  static constexpr int LDS = W_BYTES + R2;
  static constexpr bool FITS = LDS <= LDS_MAX && NPASS <= 2;
  static constexpr int BLK_PER_CU = LDS <= LDS_2BLK ? 2 : 1;
};

// AE (round 5, "accumulator epilogue"): full 8 x 16 tiles with NHWC outputs only.  The
// MFMAs run with swapped operands (A = weight rows, B = halo pixels), so a lane's
// accumulators are 4 consecutive output channels of one pixel, and the epilogue
// (bias, PReLU-input store, PReLU, residual / accumulate operand prefetched a tile
// ahead, output) goes from the accumulators straight to 8-byte stores, as in
// conv3_dense / conv3_dw: no fp32 tile through LDS and two barriers fewer per tile.
// The sums are the same MFMA k-sequence over the same operands (bit-identical).
template <int BN, int CK, bool GATE, bool AE>
__global__ __launch_bounds__(NT, 2) void conv3_ws_kernel(rdn_conv_desc d, int tiles_x, int tiles_y, int ntiles) {
  using Cfg = WsCfg<BN, CK>;
  constexpr int VEC = 8;
  constexpr int KC = Cfg::KC, WROW = Cfg::WROW, HROW = Cfg::HROW;
  constexpr int NSTEP = KC / 32;                         // MFMA k-steps of 32
  constexpr int NTL = Cfg::NTL, NTP = Cfg::NTP, NPASS = Cfg::NPASS;
  constexpr int MT = 2;                                  // 4 waves x 32 tile pixels
  constexpr int HU = CK / VEC;                           // 16-B units per halo pixel
  constexpr int H_UNITS = HW_ * HU;
  constexpr int H_IT = (H_UNITS + NT - 1) / NT;
  constexpr int CROW_F = NTP * 16 + 4;                   // epilogue fp32 row (floats)
  constexpr int UPR = BN / VEC;                          // 16-B output units per pixel
  constexpr int EU = BM * UPR;
  constexpr int E_IT = (EU + NT - 1) / NT;
  constexpr bool COLFIX = NT % UPR == 0;                 // a thread's output channels are tile-invariant
  constexpr bool KALIGN = CK % 32 == 0;                  // a k-step never straddles a tap
  constexpr bool PF = E_IT <= 6;                         // epilogue operand prefetch (register budget)
  static_assert(!GATE || NT % HU == 0, "fixed channel group per thread");
  static_assert(Cfg::FITS, "LDS");

  __shared__ __attribute__((aligned(16))) unsigned char lds[Cfg::LDS];
  unsigned char* const wl = lds;
  unsigned char* const halo = lds + Cfg::W_BYTES;
  float* const Ct = (float*)(lds + Cfg::W_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int H = d.h, W = d.w;
  const int flags = d.flags;

  // this block's tiles: XCD share [t_lo, t_hi), strided by the XCD's block count
  const int per = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7;
  const int t_hi = (int)((int64_t)ntiles * (xcd + 1) / 8);
  int t = (int)((int64_t)ntiles * xcd / 8) + (blockIdx.x >> 3);
  if (t >= t_hi) return;

  const bf16* __restrict__ X = (const bf16*)d.x;
  const bf16* __restrict__ G = (const bf16*)d.gate;

  // ---- resident weights: BN rows x KC, one load per block
  {
    const bf16* __restrict__ WP = (const bf16*)d.wp;
    constexpr int UPRW = KC / VEC;
    for (int u = tid; u < BN * UPRW; u += NT) {
      const int n = u / UPRW, k8 = u - n * UPRW;
      *(u32x4*)(wl + n * WROW + k8 * 16) = *(const u32x4*)(WP + (int64_t)n * d.kp + k8 * VEC);
    }
  }

  // ---- tile-invariant per-thread geometry, computed once: every address below is
  // a per-tile uniform base plus one of these offsets (no per-tile index math)
  // Unit order of the halo loads: pixel-major (u -> pixel, 16-B unit) for plain
  // operands; plane-major for channel-blocked ones (u -> plane, pixel, unit in the
  // plane row), so the lanes of one load instruction walk consecutive pixels of ONE
  // plane instead of scattering over every plane a pixel spans.  The LDS image is
  // the same either way.  GATE keeps one channel unit per thread (galpha).
  const int hupp = (!GATE && d.x_pl && d.x_c0 % d.x_ps == 0 && HU % (d.x_ps / VEC) == 0) ? (int)(d.x_ps / VEC) : HU;
  int hrel[H_IT], grel[GATE ? H_IT : 1], hlds[H_IT];
#pragma unroll
  for (int it = 0; it < H_IT; ++it) {
    const int u = tid + it * NT;
    const int pln = u / (HW_ * hupp), rem = u - pln * (HW_ * hupp);
    const int hp = u < H_UNITS ? rem / hupp : HW_ - 1, cu = u < H_UNITS ? pln * hupp + rem % hupp : 0;
    const int hy = hp / (TW + 2), hx = hp - hy * (TW + 2);
    hrel[it] = (hy * W + hx) * (int)d.x_ps + rdn_coff32(d.x_c0 + cu * VEC, (int)d.x_ps, (int)d.x_pl);
    if constexpr (GATE) grel[it] = (hy * W + hx) * (int)d.gate_ps + rdn_coff32(cu * VEC, (int)d.gate_ps, (int)d.gate_pl);
    hlds[it] = hp * HROW + cu * 16;
  }
  // A-operand LDS offsets per k-step (lane group g covers k = 32 j + 8 g .. +7):
  // immediates when CK is a multiple of 32, else one register per k-step
  const int a_lane = ((wave * MT) * (TW + 2) + r) * HROW;
  int offA[KALIGN ? 1 : NSTEP];
  if constexpr (!KALIGN) {
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      const int k = 32 * j + 8 * g;
      int tap = k / CK;
      const int ci = k - tap * CK;
      tap = tap < 9 ? tap : 8;   // padded k: zero weights, finite operand
      offA[j] = a_lane + ((tap / 3) * (TW + 2) + tap % 3) * HROW + ci * 2;
    }
  }
  const unsigned char* const pa = halo + (KALIGN ? a_lane + g * 16 : 0);
  const unsigned char* const pb = wl + r * WROW + g * 16;

  // output units of this thread: pixel offset within the tile (NHWC pixel index
  // relative to the tile origin) and channel
  int erel[E_IT], ecol[COLFIX ? 1 : E_IT];
#pragma unroll
  for (int it = 0; it < E_IT; ++it) {
    const int u = tid + it * NT;
    const int px = u / UPR;
    erel[it] = (px / TW) * W + px % TW;
    if constexpr (!COLFIX) ecol[it] = (u - px * UPR) * VEC;
  }
  if constexpr (COLFIX) ecol[0] = (tid % UPR) * VEC;
  auto col_of = [&](int it) { return COLFIX ? ecol[0] : ecol[it]; };
  // channel offsets of an output unit in the pre / out / residual operands
  // (channel-blocked layouts: rdn_coff); fixed per thread when COLFIX
  // (32-bit: the host checks channel-blocked offsets stay below 2^31)
  int cf_pre = 0, cf_out = 0, cf_res = 0;
  if constexpr (COLFIX) {
    cf_pre = rdn_coff32(ecol[0], (int)d.pre_ps, (int)d.pre_pl);
    cf_out = rdn_coff32(d.out_c0 + ecol[0], (int)d.out_ps, (int)d.out_pl);
    cf_res = rdn_coff32(d.res_c0 + ecol[0], (int)d.res_ps, (int)d.res_pl);
  }
  auto off_pre = [&](int c) { return COLFIX ? cf_pre : rdn_coff32(c, (int)d.pre_ps, (int)d.pre_pl); };
  auto off_out = [&](int c) { return COLFIX ? cf_out : rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl); };
  auto off_res = [&](int c) { return COLFIX ? cf_res : rdn_coff32(d.res_c0 + c, (int)d.res_ps, (int)d.res_pl); };

  // fast epilogue: whole 16-B NHWC units, no NCHW output
  const bool fast_epi = (d.ncols % VEC) == 0 && !(flags & RDN_EPI_OUT_NCHW) &&
                        (!(flags & RDN_EPI_RESID) || (d.res_climit % VEC == 0 && d.res_ps % VEC == 0 &&
                                                      d.res_c0 % VEC == 0)) &&
                        d.out_ps % VEC == 0 && d.out_c0 % VEC == 0 && d.pre_ps % VEC == 0;
  // bias / PReLU slope of a thread's fixed column, in registers (colfix); other
  // orders read them per unit (L1-resident, a few hundred bytes)
  float ebias[COLFIX ? VEC : 1], ealpha[COLFIX ? VEC : 1];
  if constexpr (COLFIX) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const int c = ecol[0] + q;
      ebias[q] = ((flags & RDN_EPI_BIAS) && c < d.ncols) ? d.bias[c] : 0.f;
      ealpha[q] = ((flags & RDN_EPI_PRELU) && c < d.ncols) ? d.alpha[c] : 0.f;
    }
  }

  float galpha[GATE ? VEC : 1];
  if constexpr (GATE) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) galpha[q] = d.gate_alpha[(tid % HU) * VEC + q];
  }

  // one tile's halo loads in flight in registers while the tile in LDS computes (a
  // second tile in flight, r02, cost occupancy and made the level-0 layers 0-20 % slower)
  constexpr int GH = GATE ? H_IT : 1;
  u32x4 hA[H_IT], gA[GH];
  auto origin = [&](int tt, int& oy, int& ox, int& on) {
    const int tx = tt % tiles_x;
    tt /= tiles_x;
    oy = (tt % tiles_y) * TH;
    ox = tx * TW;
    on = tt / tiles_y;
  };
  // every load is issued unconditionally through a buffer descriptor (out-of-image
  // units read zeros past its range): predicated flat loads became branches whose
  // vmcnt(0) waits drained the next tile's loads
  auto load_halo = [&](int oy, int ox, int on, u32x4 (&hreg)[H_IT], u32x4 (&greg)[GH]) {
    const int64_t hpix0 = ((int64_t)on * H + (oy - 1)) * W + (ox - 1);   // halo pixel (0, 0)
    const __amdgpu_buffer_rsrc_t rx = rdn_rsrc(X + hpix0 * d.x_ps);
    const __amdgpu_buffer_rsrc_t rg = rdn_rsrc(GATE ? G + hpix0 * d.gate_ps : X);
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      const int u = tid + it * NT;
      const int hp = hlds[it] / HROW;   // this unit's halo pixel (pixel- or plane-major order)
      const int hy = hp / (TW + 2), hx = hp - hy * (TW + 2);
      const bool ok = ((it + 1 < H_IT) || u < H_UNITS) & ((unsigned)(oy - 1 + hy) < (unsigned)H) &
                      ((unsigned)(ox - 1 + hx) < (unsigned)W);
#ifdef WS_DIAG_NO_LOAD   // diagnostic build: no halo loads (operands stay finite)
      (void)rx; (void)rg;
      hreg[it] = u32x4{(unsigned)ok, 0u, 0u, 0u};
      if constexpr (GATE) greg[it] = u32x4{0u, 0u, 0u, 0u};
#else
      hreg[it] = rdn_ld16(rx, ok, hrel[it] * 2);
      if constexpr (GATE) greg[it] = rdn_ld16(rg, ok, grel[it] * 2);
#endif
    }
  };
  auto store_halo = [&](const u32x4 (&hreg)[H_IT], const u32x4 (&greg)[GH]) {
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      if (it + 1 == H_IT && tid + it * NT >= H_UNITS) continue;
      u32x4 v = hreg[it];
      if constexpr (GATE) {
        float dy[VEC], pr[VEC];
        Unit16<bf16>::unpack(v, dy);
        Unit16<bf16>::unpack(greg[it], pr);
#pragma unroll
        for (int q = 0; q < VEC; ++q) dy[q] = pr[q] > 0.f ? dy[q] : galpha[q] * dy[q];
        v = Unit16<bf16>::pack(dy);
      }
      *(u32x4*)(halo + hlds[it]) = v;
    }
  };

  // epilogue read operand of a tile (residual, else the output it accumulates
  // into), loaded one tile ahead so the epilogue does not wait on a load issued
  // behind its own stores (fast epilogue, full tiles only)
  const bool pf_res = PF && fast_epi && (flags & RDN_EPI_RESID);
  const bool pf_acc = PF && fast_epi && !pf_res && (flags & RDN_EPI_ACCUM);
  u32x4 eop[PF ? E_IT : 1];
  auto load_epi = [&](int oy, int ox, int on) {
    if constexpr (!PF) return;
    if (!(pf_res || pf_acc)) return;   // launch-uniform
    const bool full = oy + TH <= H && ox + TW <= W;   // other tiles take the generic epilogue
    const int64_t opix0 = ((int64_t)on * H + oy) * W + ox;
    const int ps = pf_res ? d.res_ps : d.out_ps;
    const __amdgpu_buffer_rsrc_t rb =
        rdn_rsrc(pf_res ? (const bf16*)d.res + opix0 * d.res_ps : (const bf16*)d.out + opix0 * d.out_ps);
#pragma unroll
    for (int it = 0; it < E_IT; ++it) {
      const int c = col_of(it);
      const bool ok = full && ((it + 1 < E_IT) || tid + it * NT < EU) && c < (pf_res ? d.res_climit : d.ncols);
      eop[it] = rdn_ld16(rb, ok, (erel[it] * ps + (pf_res ? off_res(c) : off_out(c))) * 2);
    }
  };

  // ---- AE: per-lane channel offsets / bias / slope of its (n-tile, 4-channel group)s
  const bool ae_res = flags & RDN_EPI_RESID, ae_acc = flags & RDN_EPI_ACCUM;
  int ae_co[AE ? NTL : 1], ae_cp[AE ? NTL : 1], ae_ce[AE ? NTL : 1];
  bool ae_eok[AE ? NTL : 1];
  f32x4 ae_b[AE ? NTL : 1], ae_a[AE ? NTL : 1];
  f32x4 ae_b2[AE && BN <= 64 ? NTL : 1], ae_a2[AE && BN <= 64 ? NTL : 1];
  // (MT == 2: the two pixel rows of a wave pair up; up to 64 columns: the wider
  // instantiations spilled with the second bias / slope registers)
  constexpr bool W16 = AE && BN <= 64;
  if constexpr (AE) {
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) {
      const int c = jn * 16 + (W16 ? 8 * (g >> 1) : 4 * g);
      const bool in = c < d.ncols;
      ae_co[jn] = rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl);
      ae_cp[jn] = rdn_coff32(c, (int)d.pre_ps, (int)d.pre_pl);
      ae_eok[jn] = in && (ae_res ? c < d.res_climit : ae_acc);
      ae_ce[jn] = ae_res ? rdn_coff32(d.res_c0 + c, (int)d.res_ps, (int)d.res_pl) : ae_co[jn];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ae_b[jn][e] = ((flags & RDN_EPI_BIAS) && in) ? d.bias[c + e] : 0.f;
        ae_a[jn][e] = ((flags & RDN_EPI_PRELU) && in) ? d.alpha[c + e] : 0.f;
        if constexpr (W16) {   // (the unit's second half: channels c + 4 ..)
          ae_b2[jn][e] = ((flags & RDN_EPI_BIAS) && in) ? d.bias[c + 4 + e] : 0.f;
          ae_a2[jn][e] = ((flags & RDN_EPI_PRELU) && in) ? d.alpha[c + 4 + e] : 0.f;
        }
      }
    }
  }
  // (AE) residual / accumulate operand of a tile: lane (r, g) reads its 4 channels of
  // pixel (tile row 2 wave + i, column r)
  auto ae_load = [&](int oy, int ox, int on, u32x2 (&ae_eo)[MT][NTL]) {
    if constexpr (AE) {
      const int64_t opix0 = ((int64_t)on * H + oy) * W + ox;
      const int eps = ae_res ? (int)d.res_ps : (int)d.out_ps;
      const __amdgpu_buffer_rsrc_t rb =
          rdn_rsrc(ae_res ? (const bf16*)d.res + opix0 * d.res_ps : (const bf16*)d.out + opix0 * d.out_ps);
      if constexpr (W16) {   // one 16-byte unit per n-tile: [0][jn] its low, [1][jn] its high half
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) {
          const u32x4 q = rdn_ld16(rb, ae_eok[jn], (((2 * wave + (g & 1)) * W + r) * eps + ae_ce[jn]) * 2);
          ae_eo[0][jn] = u32x2{q[0], q[1]};
          ae_eo[1][jn] = u32x2{q[2], q[3]};
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          ae_eo[i][jn] = rdn_ld8(rb, ae_eok[jn], (((2 * wave + i) * W + r) * eps + ae_ce[jn]) * 2);
    }
  };
  auto ae_tile = [&](int y0, int x0, int nimg, const u32x2 (&ae_eo)[MT][NTL]) {
    f32x4 acc[MT][NTL];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int PF = 0, NB = PF + 1;
    u32x4 af[NB][MT], bfr[NB][NTL];
    auto rd = [&](int j, int b) {
      int ao;
      if constexpr (KALIGN) {
        const int k0 = 32 * j;
        int tap = k0 / CK;
        const int ci = k0 - tap * CK;
        tap = tap < 9 ? tap : 8;
        ao = ((tap / 3) * (TW + 2) + tap % 3) * HROW + ci * 2;
      } else {
        ao = offA[j];
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) af[b][i] = *(const u32x4*)(pa + ao + i * (TW + 2) * HROW);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) bfr[b][jn] = *(const u32x4*)(pb + jn * 16 * WROW + j * 64);
    };
#pragma unroll
    for (int p = 0; p < PF && p < NSTEP; ++p) rd(p, p);
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      if (j + PF < NSTEP) rd(j + PF, (j + PF) % NB);
      if constexpr (PF > 0) __builtin_amdgcn_sched_barrier(0);
      if constexpr (PF == 0) rd(j, 0);
      const int b = j % NB;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)   // D^T[m = column][n = pixel]
#ifdef WS_DIAG_NO_MFMA   // diagnostic build: fragments consumed without MFMAs
          acc[i][jn][0] += __builtin_bit_cast(float, bfr[b][jn][0] ^ af[b][i][0]);
#else
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[b][jn]),
                                                               __builtin_bit_cast(bf16x8, af[b][i]), acc[i][jn], 0,
                                                               0, 0);
#endif
    }
    const int64_t opix0 = ((int64_t)nimg * H + y0) * W + x0;
    bf16* const ob = (bf16*)d.out + opix0 * d.out_ps;
    bf16* const pb_ = (bf16*)d.pre + opix0 * d.pre_ps;
    if constexpr (W16) {
      static_assert(MT == 2, "W16 pairs the two pixel rows of a wave");
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        if (jn * 16 + 8 * (g >> 1) >= d.ncols) continue;
        // (whole-vector bit casts only: rdn_common.h's note on ext_vector elements)
        const u32x4 ua = __builtin_bit_cast(u32x4, acc[0][jn]), ub = __builtin_bit_cast(u32x4, acc[1][jn]);
        u32x4 lo, hi;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane16_swap(ua[e], ub[e], false, false);
          lo[e] = sw[0];
          hi[e] = sw[1];
        }
        const f32x4 flo = __builtin_bit_cast(f32x4, lo), fhi = __builtin_bit_cast(f32x4, hi);
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = flo[e] + ae_b[jn][e];
          v[4 + e] = fhi[e] + ae_b2[jn][e];
        }
        const int prow = (2 * wave + (g & 1)) * W + r;
        if (flags & RDN_EPI_STORE_PRE) *(u32x4*)(pb_ + prow * (int)d.pre_ps + ae_cp[jn]) = Unit16<bf16>::pack(v);
        if (flags & RDN_EPI_PRELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = v[e] > 0.f ? v[e] : ae_a[jn][e] * v[e];
            v[4 + e] = v[4 + e] > 0.f ? v[4 + e] : ae_a2[jn][e] * v[4 + e];
          }
        }
        if (ae_eok[jn]) {
          v[0] += bf16lo(ae_eo[0][jn][0]); v[1] += bf16hi(ae_eo[0][jn][0]);
          v[2] += bf16lo(ae_eo[0][jn][1]); v[3] += bf16hi(ae_eo[0][jn][1]);
          v[4] += bf16lo(ae_eo[1][jn][0]); v[5] += bf16hi(ae_eo[1][jn][0]);
          v[6] += bf16lo(ae_eo[1][jn][1]); v[7] += bf16hi(ae_eo[1][jn][1]);
        }
#ifdef WS_DIAG_NO_STORE
        if (flags & (1 << 30))
#endif
        *(u32x4*)(ob + prow * (int)d.out_ps + ae_co[jn]) = Unit16<bf16>::pack(v);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        if (jn * 16 + 4 * g >= d.ncols) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][jn][e] + ae_b[jn][e];
        const int prow = (2 * wave + i) * W + r;
        if (flags & RDN_EPI_STORE_PRE) *(u32x2*)(pb_ + prow * (int)d.pre_ps + ae_cp[jn]) = rdn_pack4(v);
        if (flags & RDN_EPI_PRELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : ae_a[jn][e] * v[e];
        }
        if (ae_eok[jn]) {
          v[0] += bf16lo(ae_eo[i][jn][0]); v[1] += bf16hi(ae_eo[i][jn][0]);
          v[2] += bf16lo(ae_eo[i][jn][1]); v[3] += bf16hi(ae_eo[i][jn][1]);
        }
#ifdef WS_DIAG_NO_STORE   // diagnostic build: no output stores (values stay live)
        if (flags & (1 << 30))
#endif
        *(u32x2*)(ob + prow * (int)d.out_ps + ae_co[jn]) = rdn_pack4(v);
      }
  };

  // the tile whose halo is in LDS: 9 taps x MFMA, then the fused epilogue
  auto compute_tile = [&](int y0, int x0, int nimg) {
    f32x4 acc[MT][NTL];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      u32x4 af[MT], bfr[NTL];
      int ao;
      if constexpr (KALIGN) {
        const int k0 = 32 * j;
        int tap = k0 / CK;
        const int ci = k0 - tap * CK;
        tap = tap < 9 ? tap : 8;
        ao = ((tap / 3) * (TW + 2) + tap % 3) * HROW + ci * 2;
      } else {
        ao = offA[j];
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *(const u32x4*)(pa + ao + i * (TW + 2) * HROW);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) bfr[jn] = *(const u32x4*)(pb + jn * 16 * WROW + j * 64);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                               __builtin_bit_cast(bf16x8, bfr[jn]), acc[i][jn], 0, 0,
                                                               0);
    }
    __syncthreads();   // halo reads done: Ct aliases it

    const bool full_tile = y0 + TH <= H && x0 + TW <= W;
    const int64_t opix0 = ((int64_t)nimg * H + y0) * W + x0;
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = p * NTP; jn < (p + 1) * NTP && jn < NTL; ++jn)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            Ct[(wave * 32 + i * 16 + g * 4 + e) * CROW_F + (jn - p * NTP) * 16 + r] = acc[i][jn][e];
      __syncthreads();
      if (fast_epi && full_tile) {
#pragma unroll
        for (int it = 0; it < E_IT; ++it) {
          const int u = tid + it * NT;
          const int c = col_of(it);
          if ((it + 1 == E_IT && u >= EU) || c < p * NTP * 16 || c >= (p + 1) * NTP * 16 || c >= d.ncols) continue;
          const int px = u / UPR;
          float v[VEC];
          const float* src = Ct + px * CROW_F + c - p * NTP * 16;
#pragma unroll
          for (int q = 0; q < VEC; q += 4) {
            const f32x4 t4 = *(const f32x4*)(src + q);
            v[q] = t4[0]; v[q + 1] = t4[1]; v[q + 2] = t4[2]; v[q + 3] = t4[3];
          }
          const int64_t opix = opix0 + erel[it];
          if (flags & RDN_EPI_BIAS) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) v[q] += COLFIX ? ebias[q] : d.bias[c + q];
          }
          if (flags & RDN_EPI_STORE_PRE) *(u32x4*)((bf16*)d.pre + opix * d.pre_ps + off_pre(c)) = Unit16<bf16>::pack(v);
          if (flags & RDN_EPI_PRELU) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
              const float a = COLFIX ? ealpha[q] : d.alpha[c + q];
              v[q] = v[q] > 0.f ? v[q] : a * v[q];
            }
          }
          bf16* const op = (bf16*)d.out + opix * d.out_ps + off_out(c);
          if (flags & (RDN_EPI_RESID | RDN_EPI_ACCUM)) {
            float rv[VEC];
            if ((flags & RDN_EPI_RESID) && c < d.res_climit) {
              Unit16<bf16>::unpack(pf_res ? eop[PF ? it : 0]
                                          : *(const u32x4*)((const bf16*)d.res + opix * d.res_ps + off_res(c)),
                                   rv);
#pragma unroll
              for (int q = 0; q < VEC; ++q) v[q] += rv[q];
            }
            if (flags & RDN_EPI_ACCUM) {
              Unit16<bf16>::unpack(pf_acc ? eop[PF ? it : 0] : *(const u32x4*)op, rv);
#pragma unroll
              for (int q = 0; q < VEC; ++q) v[q] += rv[q];
            }
          }
          *(u32x4*)op = Unit16<bf16>::pack(v);
        }
      } else {
        // ragged tile / partial units / NCHW output: generic per-unit epilogue
        c3::store_tile<bf16, NTP * 16, NT>(d, Ct, CROW_F, y0, x0, nimg, p * NTP * 16, tid);
      }
      __syncthreads();
    }

  };

  // Loads of a tile past the block's range re-read its last tile: every load is
  // issued on every path, so the compiler's vmcnt waits count exactly (a uniform
  // branch around them left it draining the other register set).
  const int t_last = t_hi - 1;
  int y0, x0, nimg;
  origin(t, y0, x0, nimg);
  if constexpr (AE) {
    // step: issue the next tile's halo and epilogue operand, this tile's MFMAs and its
    // epilogue from the accumulators, one barrier (halo consumed), the next halo to
    // LDS, one barrier (visible)
    u32x2 eC[MT][NTL], eN[MT][NTL];
    load_halo(y0, x0, nimg, hA, gA);
    store_halo(hA, gA);
    ae_load(y0, x0, nimg, eC);
    __syncthreads();
    int t1 = t + per;
    for (;;) {
      int y1 = 0, x1 = 0, n1 = 0;
      origin(min(t1, t_last), y1, x1, n1);
      load_halo(y1, x1, n1, hA, gA);
      ae_load(y1, x1, n1, eN);
      ae_tile(y0, x0, nimg, eC);
      if (t1 >= t_hi) break;
      __syncthreads();   // this tile's halo consumed by every wave
      store_halo(hA, gA);
      __syncthreads();   // next halo visible
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) eC[i][jn] = eN[i][jn];
      y0 = y1; x0 = x1; nimg = n1;
      t1 += per;
    }
    return;
  }
  load_halo(y0, x0, nimg, hA, gA);
  load_epi(y0, x0, nimg);
  store_halo(hA, gA);
  __syncthreads();
  // invariant at a step: LDS holds tile t; the next tile's (t1) loads are issued into
  // the registers before its MFMAs and stored to LDS after its epilogue
  int t1 = t + per;
  for (;;) {
    int y1 = 0, x1 = 0, n1 = 0;
    origin(min(t1, t_last), y1, x1, n1);
    load_halo(y1, x1, n1, hA, gA);   // in flight during this tile's MFMAs and epilogue
    compute_tile(y0, x0, nimg);
    if (t1 >= t_hi) break;
    load_epi(y1, x1, n1);            // in flight during the next tile's MFMAs
    store_halo(hA, gA);
    __syncthreads();
    y0 = y1; x0 = x1; nimg = n1;
    t1 += per;
  }
}

int ws_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("RDN_CONV3_WS");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on;
}

// the accumulator epilogue where it applies (RDN_WS_AE=0: the LDS-tile epilogue, for A/B)
bool ws_ae_enabled() {
  static const bool on = [] {
    const char* e = getenv("RDN_WS_AE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// resident blocks per CU of one instantiation (registers, LDS, waves), from the
// runtime's occupancy calculator, capped at 4; the persistent grid is sized to it
template <typename K>
int resident_per_cu(K kernel, int cap) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, NT, 0) != hipSuccess || n < 1) n = 1;
  return n < cap ? n : cap;
}

template <int BN, int CK, bool GATE, bool AE>
int launch_ws_k(const rdn_conv_desc* d, hipStream_t st, int tiles_x, int tiles_y, int ntiles, int cus) {
  auto kern = conv3_ws_kernel<BN, CK, GATE, AE>;
  static const int bpc = resident_per_cu(kern, 4);   // persistent blocks per CU: what is resident
  const int per_xcd = (ntiles + 7) / 8;
  int slots = cus * bpc / 8;
  if (slots > per_xcd) slots = per_xcd;
  if (slots < 1) slots = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)(8 * slots)), dim3(NT), 0, st, *d, tiles_x, tiles_y, ntiles);
  return rdn_check_launch("rdn_conv_fwd(conv3 ws)");
}

template <int BN, int CK>
int launch_ws(const rdn_conv_desc* d, hipStream_t st) {
  using Cfg = WsCfg<BN, CK>;
  if constexpr (!Cfg::FITS) {
    return 1;
  } else {
    const int tiles_x = (d->w + TW - 1) / TW, tiles_y = (d->h + TH - 1) / TH;
    const int64_t nt = (int64_t)d->n * tiles_x * tiles_y;
    if (nt >= (1ll << 31)) return 1;
    const int ntiles = (int)nt;
    {   // byte offsets of the tile-relative buffer loads stay below RDN_OOB
      const int64_t span = (int64_t)(TH + 2) * d->w;
      auto fits = [&](int64_t ps, int64_t pl, int c_hi) {
        return 2 * (span * ps + rdn_coff(c_hi, ps, pl)) < (int64_t)RDN_OOB - 16;
      };
      if (!fits(d->x_ps, d->x_pl, d->x_c0 + d->cin) || (d->gate && !fits(d->gate_ps, d->gate_pl, d->cin)) ||
          ((d->flags & RDN_EPI_RESID) && d->res && !fits(d->res_ps, d->res_pl, d->res_c0 + d->ncols)) ||
          (d->out && !fits(d->out_ps, d->out_pl, d->out_c0 + d->ncols)))
        return 1;
    }
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    static int cached_cus = 0;
    if (!cached_cus) {
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
      cached_cus = cus;
    }
    cus = cached_cus;
    constexpr int HU = CK / 8;
    if (d->gate && NT % HU != 0) return 1;
    // accumulator epilogue: full tiles, NHWC 4-channel groups, 8-byte aligned operands
    const int64_t span = (int64_t)TH * d->w;
    constexpr bool w16 = BN <= 64;
    auto ok4 = [](int64_t ps, int64_t c0, const void* p) {   // (w16: 16-byte units of 8 channels)
      return w16 ? (ps % 8 == 0 && c0 % 8 == 0 && !((uintptr_t)p & 15)) : (ps % 4 == 0 && c0 % 4 == 0 && !((uintptr_t)p & 7));
    };
    auto fit = [&](int64_t ps, int64_t pl, int c_hi) {
      return 2 * (span * ps + rdn_coff(c_hi, ps, pl)) < (int64_t)RDN_OOB - 16;
    };
    // (the gated 96-column accumulator-epilogue instantiation spilled: LDS-tile epilogue there)
    const bool ae = ws_ae_enabled() && !(d->gate && BN > 80) && d->h % TH == 0 && d->w % TW == 0 && d->ncols % (w16 ? 8 : 4) == 0 &&
                    !(d->flags & RDN_EPI_OUT_NCHW) && ok4(d->out_ps, d->out_c0, d->out) &&
                    fit(d->out_ps, d->out_pl, d->out_c0 + d->ncols) &&
                    (!(d->flags & RDN_EPI_STORE_PRE) || (ok4(d->pre_ps, 0, d->pre) && fit(d->pre_ps, d->pre_pl, d->ncols))) &&
                    (!(d->flags & RDN_EPI_RESID) ||
                     (ok4(d->res_ps, d->res_c0, d->res) && d->res_climit % (w16 ? 8 : 4) == 0 &&
                      fit(d->res_ps, d->res_pl, d->res_c0 + d->ncols)));
    RDN_PROBE("conv3_ws_kernel<bf16,%d,%d%s%s>", BN, CK, d->gate ? ",gate" : "", ae ? ",ae" : "");
    if (d->gate) {
      if constexpr (NT % HU == 0) {
        if constexpr (BN > 80) {
          return launch_ws_k<BN, CK, true, false>(d, st, tiles_x, tiles_y, ntiles, cus);
        } else {
          return ae ? launch_ws_k<BN, CK, true, true>(d, st, tiles_x, tiles_y, ntiles, cus)
                    : launch_ws_k<BN, CK, true, false>(d, st, tiles_x, tiles_y, ntiles, cus);
        }
      } else {
        return 1;
      }
    }
    return ae ? launch_ws_k<BN, CK, false, true>(d, st, tiles_x, tiles_y, ntiles, cus)
              : launch_ws_k<BN, CK, false, false>(d, st, tiles_x, tiles_y, ntiles, cus);
  }
}

template <int CK>
int ws_bn(const rdn_conv_desc* d, hipStream_t st) {
  switch ((d->ncols + 15) / 16) {
    case 1: return launch_ws<16, CK>(d, st);
    case 2: return launch_ws<32, CK>(d, st);
    case 3: return launch_ws<48, CK>(d, st);
    case 4: return launch_ws<64, CK>(d, st);
    case 5: return launch_ws<80, CK>(d, st);
    case 6: return launch_ws<96, CK>(d, st);
  }
  return 1;
}

}  // namespace

// 0 = launched, < 0 = error, 1 = shape not served here (caller uses conv3_halo)
int rdn_conv3_ws_launch(const rdn_conv_desc* d, int ck, hipStream_t st) {
  if (!ws_enabled() || d->dtype != RDN_BF16 || d->bn || ck != d->cin || d->ncols > 96 || d->gout) return 1;
  if (d->x_ps % 8 || d->x_c0 % 8 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15) || d->kp % 8) return 1;
  switch (ck) {
    case 8: return ws_bn<8>(d, st);
    case 16: return ws_bn<16>(d, st);
    case 32: return ws_bn<32>(d, st);
    case 48: return ws_bn<48>(d, st);
    case 64: return ws_bn<64>(d, st);
    case 80: return ws_bn<80>(d, st);
    case 96: return ws_bn<96>(d, st);
  }
  return 1;
}
