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
// Persistent grid, one 8-wave block per CU, XCD-local tile ranges (as conv3_ws).
// The waves split by role, so each role's registers fit two tiles of loads in
// flight (the layers are HBM-latency bound: with one tile in flight the v1 of this
// kernel spent 120 of its 200 us in the load -> barrier chain, measured with the
// MFMAs and stores switched off):
//
//   waves 0-3 (D): gated dY halo loads (+ the PReLU-backward gate and dalpha/dbias
//     partials on the way to LDS), dgrad MFMAs (32 pixels x BN per wave), the dX
//     epilogue (residual / accumulate operand prefetched one tile ahead);
//   waves 4-7 (W): X halo loads, wgrad MFMAs (n-tiles w, w+4, ...), accumulators in
//     registers over the block's tiles; ONE split-K slab per block at the end
//     (split = block), summed with the partials by rdn_wgrad_reduce in fixed order.
//
// Every global load in the tile loop is unconditional (out-of-image units read a
// zero line), so the compiler's vmcnt waits count exactly and the wait for tile
// t+1 does not drain tile t+2's loads.
//
// Column halves (NH = 2, round 4): the level-1 conv_1 / conv_2 (96 / 128 input
// channels, 32 dY channels) in one pass as well.  A block serves one half of the
// input channels, [col0, col0 + BN) with BN = ncols / 2, for every tile of its range:
// its dX slice, the matching rows of the resident weight panel, its X channels and
// its weight-gradient columns (tap, ci in the half: a slab of mdim x 9*BN, the
// blocks of half h at slabs [h*G/2, (h+1)*G/2), summed by rdn_wgrad_reduce_cols).
// Both halves gate the same dY tile; only half 0 counts the dalpha / dbias partials
// (half 1 writes zero rows).  The whole 96 / 128-column tile would not fit: the
// resident panel and the W waves' accumulators grow with the columns (<96,32>
// spilled, r02).
//
// Gate-out (GO, round 4; d.gout as in conv3_big): when this conv is the last consumer
// (in backward order) of another layer's output and that output is the tail
// [gout_c0, ncols) of its input channels, the dX of those channels is that layer's
// complete dY: the D waves' epilogue gates it with the layer's saved PReLU input
// (prefetched one tile ahead beside the accumulate operand) and stores its dYpre
// instead, summing the layer's dalpha / dbias partials in registers; one partial row
// per block (= per slab; zeros in the columns of the other half); with
// RDN_EPI_GOUT_KEEP the dY is stored as well (a block's conv_3 reads its own output
// gradient again as the residual operand of its input gradient).  Served for
// up_0.conv (finishes up_0.conv_t: <48,32,h2>, gout_c0 = 32) and the level-1
// conv_0s (finish down_0 / block_1_k.conv_3: <64,32>, gout_c0 = 0), whose separate
// PReLU-backward passes (73 / 23 us each at B16) leave the compute queue.
#include "conv3_tile.h"

#include <stdlib.h>

namespace {

using c3::BM;
using c3::HW_;
using c3::TH;
using c3::TW;

constexpr int NT = 512;   // 8 waves
// Schedule (each choice measured per launch and on the step; DESIGN.md sections 9-10):
//  * weight-gradient fragments prefetched 3 (k-step, n-tile) steps ahead;
//  * one barrier per tile (dY and X halos double-buffered in LDS) where it measured faster;
//  * on the level-0 one-barrier shapes the W waves load and gate the dY halo ring and the
//    D waves the tile interior (the D waves are the critical path of a tile);
//  * dX epilogue in 16-byte units (lane-row swap by v_permlane16_swap) except gate-out;
//  * the pre-gated 64-channel dY halo of the five-part level-1 conv_3 (h5) arrives by
//    LDS-DMA (dense 128-B pixel rows; physical 16-B unit pu of halo column hx holds logical
//    unit pu ^ (hx & 7): both fragment reads conflict-free by exhaustive model), into THREE
//    buffers (the DMA of tile t + 2 per issued after tile t's epilogue, so it has a whole
//    step to land), and h5's D waves hold the whole 32-column dgrad weight panel in VGPRs
//    (144 registers per lane), waited for before the tile loop.
//    Per launch at B16 / B32 (profiles/r05_ddma_kbench_ab.txt, r05_wreg_kbench_ab.txt,
//    r05_h5_d3_kbench.txt): 112.0 -> 105.8 -> 99.0 -> 92.8 us / 210 -> 197 -> 185 -> 189 us.
constexpr int DW_WPIPE = 3;   // weight-gradient fragment prefetch depth
constexpr int LDS_MAX = 160 * 1024;

__device__ __attribute__((aligned(64))) unsigned int g_dw_zero[16];

template <int N>
__device__ __forceinline__ void dw_wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// one LDS-DMA wave-instruction: 16 B per lane from `src` to LDS byte dst + lane*16 (dst
// wave-uniform, in M0; inline asm, so the compiler does not count it on its waits --
// the step's explicit vmcnt wait before the barrier is the ordering, as in conv3_big)
__device__ __forceinline__ void dw_glds16(const void* src, unsigned dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}
__device__ __forceinline__ unsigned dw_lds_addr(const unsigned char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

#ifdef DW_STAMPS
// diagnostic build: per wave, cycles (s_memtime) spent in each phase of the tile loop,
// summed over the block's tiles of the last launch: [block][wave][phase 0..5, tiles, -]
__device__ unsigned long long g_dw_st[512 * 8 * 8];
#define DW_NOW() __builtin_amdgcn_s_memtime()
#endif

template <int BN, int CK, bool GO = false, bool DDMA_ = false>
struct DwCfg {
  static constexpr int KC = (9 * CK + 63) / 64 * 64;   // packed dgrad K (rdn_pack_weights, conv3_ws)
  static constexpr int NSTEP = KC / 32;
  static constexpr int WROW = KC * 2 + 32;              // = 32 mod 128: conflict-free B reads
  static constexpr bool DDMA = DDMA_;                   // dense swizzled rows, 1-KB DMA pieces
  static constexpr int WREGS = (KC / 32) * (BN / 16) * 4;     // panel registers per D lane
  // the register panel on h5 only: on the other shapes it measured within noise (their D
  // waves are bound by the load path, not LDS reads) and three spilled
  static constexpr bool WREG = !GO && DDMA && BN == 32;
  static constexpr int W_BYTES = WREG ? 0 : BN * WROW;
  static_assert(!DDMA || (CK == 64 && !GO), "LDS-DMA dY halo: 8 units per pixel row");
  static constexpr int DROW = DDMA ? CK * 2 : c3::HaloRow<CK * 2>::V;   // dY halo row stride (b128 and tr16 conflict-free)
  static constexpr int XROW = c3::HaloRow<BN * 2>::V;   // X halo row stride
  static constexpr bool D3 = WREG;                      // three dY halo buffers (h5)
  static constexpr int D_PIECES = D3 ? ((HW_ * CK * 2 + 1023) / 1024 + 3) / 4 * 4 : (HW_ * CK * 2 + 1023) / 1024;
  static constexpr int D_BYTES = DDMA ? D_PIECES * 1024 : (HW_ * DROW + 15) / 16 * 16;
  static constexpr int X_BYTES = (HW_ * XROW + 15) / 16 * 16;
  static constexpr int CT_BYTES = 0;                    // dX leaves from the accumulators
  static constexpr bool SB_ = !((BN == 64 && CK == 16) || (BN == 32 && CK == 32));
  // W waves gate the dY halo ring (BSPLIT below) on the level-0 shapes: per launch at B16
  // (scripts/dw_kbench.py, profiles/r05_wsh_kbench_ab.txt) 32->16 57.0 -> 55.0 us, 80->32
  // 136.4 -> 133.5, up_0.conv (h2, go) 243.9 -> 208.5; the level-1 shapes ran 1-2 us slower
  // with it (64->32 34.1 -> 35.6, h2 46.8 / 52.9 -> 47.7 / 54.4, go 46.5 -> 48.9) and h5
  // even: off there
  static constexpr bool WSH = SB_ && (CK == 16 || BN == 80 || (GO && BN == 48));
  static_assert(!DDMA || (SB_ && !WSH), "LDS-DMA dY halo: the one-barrier schedule, D waves only");
  static constexpr int RED_BYTES = 2 * (WSH ? 512 : 256) * 8 * 4;   // dalpha/dbias partial reduction (aliases)
  static constexpr int AL_BYTES = (CK * 4 + 15) / 16 * 16;   // gate slopes
  static constexpr int GAL_BYTES = GO ? BN * 4 : 0;           // gate-out: the finished layer's slopes
  // W waves keep two X halos in flight in registers where the budget allows it
  // (accumulators MTW x NTW x 4 + two X_IT sets within 256 VGPRs at 2 waves/SIMD);
  // otherwise ONE register set and two X halo buffers in LDS
  static constexpr int X_IT = (HW_ * (BN / 8) + 255) / 256;
  static constexpr int NTW = (9 * BN / 16 + 3) / 4;
  static constexpr bool DW2 = (CK / 16) * NTW * 4 + 2 * X_IT * 4 <= 112;
  // single-barrier schedule: both halos double-buffered in LDS, the D waves' gate
  // pass overlapping the W waves' MFMAs (per launch, profiles/r03_v15_dw_sb_kbench:
  // 32->16 59 -> 54 us, 80->32 135 -> 133, 64->32 36 -> 34; the 64->16 and 32->32
  // shapes ran 1-3 us slower and keep two barriers per tile)
  static constexpr bool SB = SB_;
  static constexpr int DB = D3 ? 3 : SB ? 2 : 1;
  static constexpr int BASE = W_BYTES + DB * D_BYTES + CT_BYTES + AL_BYTES + GAL_BYTES;
  // X halo buffers in LDS: 2 for the LDS double buffer, 1 where it would not fit
  // (96 columns were tried: <96,32> spills 128 B in the W loop, so they stay on the
  // separate kernels)
  static constexpr int XB = SB ? 2 : DW2 ? 1 : (BASE + 2 * X_BYTES <= LDS_MAX ? 2 : 1);
  // 16 B per thread of a role: the padding units of the last halo load round store
  // here instead of skipping their store (a lane-divergent skip made hipcc wait
  // vmcnt(0) at the loop head, i.e. on the previous tile's dX stores)
  static constexpr int DUMP_BYTES = 256 * 16;
  static constexpr int LDS = BASE + XB * X_BYTES + DUMP_BYTES;
  static constexpr bool FITS = LDS <= LDS_MAX && DB * D_BYTES + XB * X_BYTES + CT_BYTES >= RED_BYTES &&
                              (!GO || W_BYTES >= 8 * BN * 4);   // gate-out partials in the dead panel
};

template <int BN, int CK, int NH, bool GO, bool GT>
__global__ __launch_bounds__(NT, 1) void conv3_dw_kernel(rdn_conv_desc d, rdn_wgrad_desc wg, int tiles_x, int tiles_y,
                                                         int ntiles) {
  using Cfg = DwCfg<BN, CK, GO, !GT && CK == 64 && !GO>;
  constexpr bool DDMA = Cfg::DDMA;
  constexpr int VEC = 8;
  constexpr int KC = Cfg::KC, NSTEP = Cfg::NSTEP, WROW = Cfg::WROW, DROW = Cfg::DROW, XROW = Cfg::XROW;
  constexpr int NR = 256;                               // threads per role
  constexpr int MT = 2;                                 // dgrad: 2 x 16 pixels per D wave
  constexpr int NTL = BN / 16;                          // dgrad n-tiles
  constexpr int NE = NTL;                               // epilogue operands per row
  constexpr int DU = CK / VEC, XU = BN / VEC;           // 16-B units per halo pixel
  constexpr int D_UNITS = HW_ * DU, X_UNITS = HW_ * XU;
  constexpr int D_IT = (D_UNITS + NR - 1) / NR, X_IT = (X_UNITS + NR - 1) / NR;
  // dY halo units of the D waves: all, or (WSH) all but the last partial round [DN, D_UNITS),
  // which the W waves take (one unit per W thread)
  constexpr bool WSH = Cfg::WSH;
  // BSPLIT: the D waves take exactly the tile-interior units (TH x TW pixels: 1 or 2
  // whole rounds at 16 / 32 dY channels) and the W waves the halo ring (52 pixels), so
  // only the D waves count dalpha / dbias partials and the W waves gate with the packed
  // form (no partial registers: the 80-column W waves spilled with them)
  constexpr int IU = TH * TW * DU;
  constexpr bool BSPLIT = WSH && IU % NR == 0 && D_UNITS - IU <= NR;
  constexpr int D_ITD = BSPLIT ? IU / NR : WSH ? D_IT - 1 : D_IT, DN = D_ITD * NR;
  constexpr int RED_T = WSH ? 2 * NR : NR;              // threads with dalpha/dbias partials
  static_assert(!WSH || (D_ITD >= 1 && D_UNITS - DN <= NR), "W share geometry");
  constexpr int MTW = CK / 16;                          // wgrad m-tiles
  constexpr int NT_ALL = 9 * BN / 16;                   // wgrad n-tiles
  constexpr int NTW = (NT_ALL + 3) / 4;                 // per W wave (n-tile = wave + 4 j)
  constexpr bool KALIGN = CK % 32 == 0;                 // a dgrad k-step never straddles a tap
  constexpr int RS = (TW + 2);                          // halo pixels per halo row
  static_assert(NR % DU == 0, "fixed dY channel group per thread");
  static_assert(BN % 16 == 0 && CK % 16 == 0, "16-wide MFMA tiles");
  static_assert(Cfg::FITS, "LDS");
  constexpr bool DW2 = Cfg::DW2;
  static_assert(Cfg::X_IT == X_IT && Cfg::NTW == NTW, "cfg");

  __shared__ __attribute__((aligned(16))) unsigned char lds[Cfg::LDS];
  unsigned char* const wl = lds;
  unsigned char* const dyh = lds + Cfg::W_BYTES;
  unsigned char* const xh = dyh + Cfg::DB * Cfg::D_BYTES;
  float* const alds = (float*)(xh + Cfg::XB * Cfg::X_BYTES + Cfg::CT_BYTES);
  unsigned char* const dump = lds + Cfg::LDS - Cfg::DUMP_BYTES;
  float* const galds = alds + Cfg::AL_BYTES / 4;        // (GO) slopes of the finished layer, this half's columns
  float* const gred = (float*)lds;                      // (GO) its partials, [D wave][2][BN] over the dead panel
  float* const red = (float*)(lds + Cfg::W_BYTES);   // partial reduction (aliases the halos after the loops)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool dwave = wave < 4;                          // role (wave-uniform)
#ifdef DW_STAMPS
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_mid = 0;
#endif
  const int rt = tid & (NR - 1), rw = wave & 3;         // thread / wave within the role
  const int r = lane & 15, g = lane >> 4;
  const int H = d.h, W = d.w;
  const int flags = d.flags;

  // this block's tiles: XCD share, strided by the XCD's block count (conv3_ws); with
  // column halves the XCD's blocks alternate halves and each half strides its own
  const int per = (gridDim.x >> 3) / NH;
  const int xcd = blockIdx.x & 7;
  const int jb = blockIdx.x >> 3;
  const int half = NH > 1 ? jb % NH : 0;
  const int col0 = half * BN;                           // first input channel of this block's half
  // weight-gradient slab / partial row of this block (halves: grouped by half)
  const int slab = NH > 1 ? half * (gridDim.x / NH) + xcd * per + jb / NH : (int)blockIdx.x;
  const int t_lo = (int)((int64_t)ntiles * xcd / 8);
  const int t_hi = (int)((int64_t)ntiles * (xcd + 1) / 8);
  int t = t_lo + jb / NH;
  const int t_last = t_hi - 1;                          // loads of a tile past the range re-read this one

  const bf16* __restrict__ DY = (const bf16*)d.x;
  const bf16* __restrict__ PR = (const bf16*)d.gate;
  const bf16* __restrict__ XS = (const bf16*)wg.b;

  // ---- resident dgrad weight panel: BN rows x KC
  {
    const bf16* __restrict__ WP = (const bf16*)d.wp;
    constexpr int UPRW = KC / VEC;
    for (int u = tid; u < (Cfg::WREG ? 0 : BN * UPRW); u += NT) {
      const int n = u / UPRW, k8 = u - n * UPRW;
      *(u32x4*)(wl + n * WROW + k8 * 16) = *(const u32x4*)(WP + (int64_t)(col0 + n) * d.kp + k8 * VEC);
    }
    if constexpr (GT)
      for (int c = tid; c < CK; c += NT) alds[c] = d.gate_alpha[c];
    if constexpr (GO) {
      for (int c = tid; c < BN; c += NT) {
        const int gc = col0 + c - d.gout_c0;
        galds[c] = gc >= 0 ? d.gout_alpha[gc] : 0.f;
      }
    }
  }
  __syncthreads();   // the gate slopes are read by the first halo store (before the prologue barrier)

  auto origin = [&](int tt, int& oy, int& ox, int& on) {
    const int tx = tt % tiles_x;
    tt /= tiles_x;
    oy = (tt % tiles_y) * TH;
    ox = tx * TW;
    on = tt / tiles_y;
  };
  // halo unit inside the image (pure VALU: a uniform short cut here made the compiler
  // unswitch the loads into branches with vmcnt(0) waits)
  auto in_img = [&](int hp, int oy, int ox) {
    const int hy = hp / RS, hx = hp - (hp / RS) * RS;
    return (hp < HW_) & ((unsigned)(oy - 1 + hy) < (unsigned)H) & ((unsigned)(ox - 1 + hx) < (unsigned)W);
  };

  // The two roles run separate loops (their loop-carried registers do not overlap)
  // with the same barriers per tile.  At the top of a step LDS holds tile t and the
  // register set `cur` holds tile t + per in flight; the step issues t + 2 per into
  // `nxt` (past the range it re-reads the last tile: every load is unconditional).
  if (dwave) {
    // ================= D waves: gated dY halo, dgrad, dX epilogue
    const int dcu = rt % DU;
    int lrel[D_ITD], grel[D_ITD], llds[D_ITD], uhp[D_ITD];
    unsigned dint = 0;   // bit it: unit `it` is a tile-interior pixel (counted in the partials)
#pragma unroll
    for (int it = 0; it < D_ITD; ++it) {
      const int u = rt + it * NR;
      int hp = u < D_UNITS ? u / DU : HW_;
      if constexpr (BSPLIT) hp = (hp / TW + 1) * RS + hp % TW + 1;   // interior pixel u / DU
      const int hq = hp < HW_ ? hp : 0;
      const int hy = hq / RS, hx = hq - hy * RS;
      uhp[it] = hp;
      lrel[it] = (hy * W + hx) * (int)d.x_ps + rdn_coff32(d.x_c0 + dcu * VEC, (int)d.x_ps, (int)d.x_pl);
      grel[it] = (hy * W + hx) * (int)d.gate_ps + rdn_coff32(dcu * VEC, (int)d.gate_ps, (int)d.gate_pl);
      llds[it] = hq * DROW + dcu * 16;
      if (hp < HW_ && hy >= 1 && hy <= TH && hx >= 1 && hx <= TW) dint |= 1u << it;
    }
    // (DDMA) dY halo piece pc = rw + 4 j (1 KB): halo bytes pc * 1024 + lane * 16 ->
    // pixel hp, physical unit pu = lane & 7 holding logical unit pu ^ (hx & 7);
    // out-of-image pixels (and the pad past the halo) read the zero line
    constexpr int DPW = DDMA ? (Cfg::D_PIECES + 3) / 4 : 1;
    int prel[DPW], php[DPW];
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int hp = (rw + 4 * j) * 8 + (lane >> 3);
      const int hq = hp < HW_ ? hp : 0;
      const int hy = hq / RS, hx = hq - hy * RS;
      php[j] = hp;
      prel[j] = (hy * W + hx) * (int)d.x_ps +
                rdn_coff32(d.x_c0 + ((lane & 7) ^ (hx & 7)) * VEC, (int)d.x_ps, (int)d.x_pl);
    }
    auto issue_d = [&](int tt, int doff) {
      int oy, ox, on;
      origin(tt, oy, ox, on);
      const bf16* const db = DY + (((int64_t)on * H + (oy - 1)) * W + (ox - 1)) * d.x_ps;
      const unsigned dst = dw_lds_addr(dyh) + doff;
#pragma unroll
      for (int j = 0; j < DPW; ++j) {
        const int pc = rw + 4 * j;
        if (pc >= Cfg::D_PIECES) break;   // wave-uniform
        const void* src = in_img(php[j], oy, ox) ? (const void*)(db + prel[j]) : (const void*)g_dw_zero;
        dw_glds16(src, dst + pc * 1024);
      }
    };
    float sa[VEC], sb[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      sa[q] = 0.f;
      sb[q] = 0.f;
    }
    // dX epilogue straight from the accumulators: the dgrad MFMA runs with swapped
    // operands (A = weights, B = dY), so a lane holds 4 consecutive input channels
    // jn*16 + 4g .. +3 of pixel (tile row 2 rw + i, column r) -- one 8-byte store per
    // (i, jn), no fp32 tile in LDS.  The operand: residual (channels < res_climit)
    // or the accumulated output, prefetched one tile ahead.
    const bool has_res = flags & RDN_EPI_RESID, has_acc = flags & RDN_EPI_ACCUM;
    const bf16* const ebase = has_res ? (const bf16*)d.res : (const bf16*)d.out;
    const int eps = has_res ? (int)d.res_ps : (int)d.out_ps;
    // W16 (round 5, every non-gate-out shape): the two pixel rows' accumulators are
    // exchanged between lane rows g, g^1 (v_permlane16_swap), so lane (r, g) holds 8
    // consecutive channels jn*16 + 8 (g >> 1) .. +7 of pixel (tile row 2 rw + (g & 1),
    // column r): the epilogue operand and dX move as ONE 16-byte load / store per n-tile
    // instead of two 8-byte ones (stamped diagnostic builds: the D waves spent ~1.5k
    // cycles per tile issuing the 8-byte epilogue loads, the critical path of the kernel)
    constexpr bool W16 = !GO;
    int coff_e[NTL], coff_o[NTL], coff_g[NTL];
    bool eok[NTL], gon[NTL];
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) {
      const int c = col0 + jn * 16 + (W16 ? 8 * (g >> 1) : 4 * g);
      eok[jn] = has_res ? c < d.res_climit : has_acc;
      coff_e[jn] = has_res ? rdn_coff32(d.res_c0 + c, (int)d.res_ps, (int)d.res_pl)
                           : rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl);
      coff_o[jn] = rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl);
      gon[jn] = GO && c >= d.gout_c0;   // (a 4-channel unit is wholly in or out: gout_c0 % 4 == 0)
      coff_g[jn] = gon[jn] ? c - d.gout_c0 : 0;
    }
    // (GO) the finished layer's dalpha / dbias partials of this thread's channels
    float gsa[GO ? NTL : 1][4], gsb[GO ? NTL : 1][4];
#pragma unroll
    for (int jn = 0; jn < (GO ? NTL : 1); ++jn)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gsa[jn][e] = 0.f;
        gsb[jn][e] = 0.f;
      }
    auto load = [&](int tt, u32x4 (&lr)[D_ITD], u32x4 (&gr)[D_ITD]) {
      int oy, ox, on;
      origin(tt, oy, ox, on);
      const int64_t hpix0 = ((int64_t)on * H + (oy - 1)) * W + (ox - 1);
      const __amdgpu_buffer_rsrc_t rd = rdn_rsrc(DY + hpix0 * d.x_ps);
      const __amdgpu_buffer_rsrc_t rg = rdn_rsrc(GT ? PR + hpix0 * d.gate_ps : DY);
#pragma unroll
      for (int it = 0; it < D_ITD; ++it) {
        const bool ok = in_img(uhp[it], oy, ox);
        lr[it] = rdn_ld16(rd, ok, lrel[it] * 2);
        if constexpr (GT) gr[it] = rdn_ld16(rg, ok, grel[it] * 2);
        else gr[it] = u32x4{0u, 0u, 0u, 0u};
      }
    };
    // registers -> LDS with the PReLU-backward gate and the dalpha/dbias partials of
    // the tile-interior pixels (each image pixel is interior to exactly one tile)
    auto store = [&](const u32x4 (&lr)[D_ITD], const u32x4 (&gr)[D_ITD], bool live, int doff) {
      if constexpr (!GT) {   // the operand is dYpre already (gate-out finisher / PReLU pass)
#pragma unroll
        for (int it = 0; it < D_ITD; ++it)
          *(u32x4*)(uhp[it] < HW_ ? dyh + doff + llds[it] : dump + rt * 16) = lr[it];
        return;
      }
      const f32x4 a0 = *(const f32x4*)(alds + dcu * VEC), a1 = *(const f32x4*)(alds + dcu * VEC + 4);
      if (!live) {   // (block-uniform) no partials to count: the packed gate, ~half the VALU
#pragma unroll
        for (int it = 0; it < D_ITD; ++it) {
          u32x4 o;
          o[0] = rdn_gate2(lr[it][0], gr[it][0], a0[0], a0[1]);
          o[1] = rdn_gate2(lr[it][1], gr[it][1], a0[2], a0[3]);
          o[2] = rdn_gate2(lr[it][2], gr[it][2], a1[0], a1[1]);
          o[3] = rdn_gate2(lr[it][3], gr[it][3], a1[2], a1[3]);
          *(u32x4*)(uhp[it] < HW_ ? dyh + doff + llds[it] : dump + rt * 16) = o;
        }
        return;
      }
#pragma unroll
      for (int it = 0; it < D_ITD; ++it) {
        float dy[VEC], pr[VEC];
        Unit16<bf16>::unpack(lr[it], dy);
        Unit16<bf16>::unpack(gr[it], pr);
        const bool in = live && ((dint >> it) & 1u);   // a re-read past the range counts nothing
        unsigned char* const dst = uhp[it] < HW_ ? dyh + doff + llds[it] : dump + rt * 16;
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const bool pos = pr[q] > 0.f;
          if (in && !pos) sa[q] += pr[q] * dy[q];
          dy[q] = pos ? dy[q] : (q < 4 ? a0[q] : a1[q - 4]) * dy[q];
          if (in) sb[q] += dy[q];
        }
        *(u32x4*)dst = Unit16<bf16>::pack(dy);
      }
    };
    auto load_epi = [&](int tt, u32x2 (&eo)[MT][NE]) {
      int oy, ox, on;
      origin(tt, oy, ox, on);
      const int64_t opix0 = ((int64_t)on * H + oy) * W + ox;
      const __amdgpu_buffer_rsrc_t rb = rdn_rsrc(ebase + opix0 * eps);
      if constexpr (W16) {   // one 16-byte unit per n-tile: eo[0][jn] its low, eo[1][jn] its high half
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) {
          const u32x4 q = rdn_ld16(rb, eok[jn], (((2 * rw + (g & 1)) * W + r) * eps + coff_e[jn]) * 2);
          eo[0][jn] = u32x2{q[0], q[1]};
          eo[1][jn] = u32x2{q[2], q[3]};
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          eo[i][jn] = rdn_ld8(rb, eok[jn], (((2 * rw + i) * W + r) * eps + coff_e[jn]) * 2);
    };
    // fragments: pixel r of tile rows 2 rw (+1); k-step j covers k = 32 j + 8 g
    const int a_lane = (2 * rw * RS + r) * DROW;
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
    const unsigned char* const pda = dyh + (DDMA ? (2 * rw * RS + r) * DROW : KALIGN ? a_lane + g * 16 : 0);
    // (DDMA) in-row byte offset of the lane's unit ci / 8 + g at halo column r + dx
    int dsw[DDMA ? 3 : 1][DDMA ? 2 : 1];
    if constexpr (DDMA) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int c = 0; c < 2; ++c) dsw[dx][c] = dx * DROW + (((4 * c + g) ^ ((r + dx) & 7)) * 16);
    }
    const unsigned char* const pdb = wl + r * WROW + g * 16;
    // (WREG) the lane's B fragments of every k-step: weight row col0 + 16 jn + r, k 32 j + 8 g
    u32x4 wreg[Cfg::WREG ? NSTEP : 1][Cfg::WREG ? NTL : 1];
    if constexpr (Cfg::WREG) {
      const bf16* __restrict__ WP = (const bf16*)d.wp;
#pragma unroll
      for (int j = 0; j < NSTEP; ++j)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          wreg[j][jn] = *(const u32x4*)(WP + (int64_t)(col0 + jn * 16 + r) * d.kp + j * 32 + g * 8);
      // consumed here, before the tile loop: otherwise hipcc counts these loads as pending
      // at the loop's first MFMAs and its vmcnt waits there (down to vmcnt(2)) also drain
      // the halo DMA and epilogue loads in flight on every later tile
#pragma unroll
      for (int j = 0; j < NSTEP; ++j)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) asm volatile("" : "+v"(wreg[j][jn]));
    }
    auto dgrad_tile = [&](int tt, const u32x2 (&eo)[MT][NE], int doff) {
      f32x4 acc[MT][NTL];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
      // (GO) the finished layer's PReLU input at the gated units, issued before the
      // MFMAs (prefetched a tile ahead beside `eo` instead: up_0.conv 227 -> 240 us, the
      // level-1 conv_0 spilled; loaded after the MFMAs: no spill on <64,32,go> but 4-7 %
      // longer per launch, profiles/r05_spill_layers.txt)
      u32x2 gp[GO ? MT : 1][GO ? NTL : 1];
      auto load_gp = [&]() {
        int oy, ox, on;
        origin(tt, oy, ox, on);
        const __amdgpu_buffer_rsrc_t rp =
            rdn_rsrc((const bf16*)d.gout_pre + (((int64_t)on * H + oy) * W + ox) * d.gout_pre_ps);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int jn = 0; jn < NTL; ++jn)
            gp[i][jn] = rdn_ld8(rp, gon[jn], (((2 * rw + i) * W + r) * (int)d.gout_pre_ps + coff_g[jn]) * 2);
      };
      if constexpr (GO) load_gp();
      auto aoff_of = [&](int j) {
        if constexpr (DDMA) {
          const int k0 = 32 * j, tap = k0 / CK, ci = k0 - tap * CK;
          return (tap / 3) * RS * DROW + dsw[tap % 3][ci / 32];
        } else if constexpr (KALIGN) {
          const int k0 = 32 * j;
          int tap = k0 / CK;
          const int ci = k0 - tap * CK;
          tap = tap < 9 ? tap : 8;
          return ((tap / 3) * RS + tap % 3) * DROW + ci * 2;
        } else {
          return offA[j];
        }
      };
      // (the next k-step's fragments read before the current MFMAs measured no faster on
      // any shape and spilled <64,32,go>, profiles/r05_xdma_dpf_kbench)
#pragma unroll
      for (int j = 0; j < NSTEP; ++j) {
        const int ao = aoff_of(j);
        u32x4 fa[MT], fb[NTL];
#pragma unroll
        for (int i = 0; i < MT; ++i) fa[i] = *(const u32x4*)(pda + doff + ao + i * RS * DROW);
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
          fb[jn] = Cfg::WREG ? wreg[Cfg::WREG ? j : 0][Cfg::WREG ? jn : 0] : *(const u32x4*)(pdb + jn * 16 * WROW + j * 64);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int jn = 0; jn < NTL; ++jn)   // D^T[m = column][n = pixel]
            acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[jn]),
                                                                 __builtin_bit_cast(bf16x8, fa[i]), acc[i][jn], 0,
                                                                 0, 0);
      }
#ifdef DW_STAMPS
      st_mid = DW_NOW();
#endif
      int oy, ox, on;
      origin(tt, oy, ox, on);
      bf16* const ob = (bf16*)d.out + (((int64_t)on * H + oy) * W + ox) * d.out_ps;
      if constexpr (W16) {
        static_assert(MT == 2, "W16 pairs the two pixel rows of a D wave");
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) {
          // (whole-vector bit casts only: rdn_common.h's note on ext_vector elements)
          const u32x4 ua = __builtin_bit_cast(u32x4, acc[0][jn]), ub = __builtin_bit_cast(u32x4, acc[1][jn]);
          u32x4 lo, hi;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane16_swap(ua[e], ub[e], false, false);
            lo[e] = sw[0];   // channels c + e
            hi[e] = sw[1];   // channels c + 4 + e
          }
          const f32x4 flo = __builtin_bit_cast(f32x4, lo), fhi = __builtin_bit_cast(f32x4, hi);
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = flo[e];
            v[4 + e] = fhi[e];
          }
          if (eok[jn]) {
            v[0] += bf16lo(eo[0][jn][0]); v[1] += bf16hi(eo[0][jn][0]);
            v[2] += bf16lo(eo[0][jn][1]); v[3] += bf16hi(eo[0][jn][1]);
            v[4] += bf16lo(eo[1][jn][0]); v[5] += bf16hi(eo[1][jn][0]);
            v[6] += bf16lo(eo[1][jn][1]); v[7] += bf16hi(eo[1][jn][1]);
          }
          *(u32x4*)(ob + ((2 * rw + (g & 1)) * W + r) * (int)d.out_ps + coff_o[jn]) = Unit16<bf16>::pack(v);
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) {
          float v[4] = {acc[i][jn][0], acc[i][jn][1], acc[i][jn][2], acc[i][jn][3]};
          if (eok[jn]) {
            v[0] += bf16lo(eo[i][jn][0]); v[1] += bf16hi(eo[i][jn][0]);
            v[2] += bf16lo(eo[i][jn][1]); v[3] += bf16hi(eo[i][jn][1]);
          }
          if constexpr (GO) {
            if (gon[jn]) {   // complete dY of the finished layer: its dYpre (aten prelu backward)
              if (flags & RDN_EPI_GOUT_KEEP)   // (and dY itself: that layer's residual epilogue reads it)
                *(u32x2*)(ob + ((2 * rw + i) * W + r) * (int)d.out_ps + coff_o[jn]) = rdn_pack4(v);
              const f32x4 al = *(const f32x4*)(galds + jn * 16 + 4 * g);
              const float pr[4] = {bf16lo(gp[i][jn][0]), bf16hi(gp[i][jn][0]), bf16lo(gp[i][jn][1]),
                                   bf16hi(gp[i][jn][1])};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const bool pos = pr[e] > 0.f;
                if (!pos) gsa[jn][e] += pr[e] * v[e];
                v[e] = pos ? v[e] : al[e] * v[e];
                gsb[jn][e] += v[e];
              }
              bf16* const gb = (bf16*)d.gout + (((int64_t)on * H + oy) * W + ox) * d.gout_ps;
              *(u32x2*)(gb + ((2 * rw + i) * W + r) * (int)d.gout_ps + coff_g[jn]) = rdn_pack4(v);
              continue;
            }
          }
          *(u32x2*)(ob + ((2 * rw + i) * W + r) * (int)d.out_ps + coff_o[jn]) = rdn_pack4(v);
        }
    };

    u32x4 lA[D_ITD], gA[D_ITD], lB[D_ITD], gB[D_ITD];
    u32x2 eC[MT][NE], eN[MT][NE];
    if constexpr (Cfg::SB) {
    // step k computes tile t from buffer k&1 while it gates tile t + per (issued one
    // step earlier) into buffer (k+1)&1 and issues tile t + 2 per: ONE barrier per
    // tile, and the gate pass overlaps the W waves' MFMAs instead of idling them (two
    // register sets in flight measured no faster and spill the 80-column shape)
    if (t < t_hi) {
      if constexpr (DDMA) {
        static_assert(Cfg::D3, "the LDS-DMA dY halo runs three buffers");
        issue_d(t, 0);
        issue_d(min(t + per, t_last), Cfg::D_BYTES);
        load_epi(t, eC);
        dw_wait_vm<0>();
      } else {
        load(t, lA, gA);
        store(lA, gA, half == 0, 0);
        load(min(t + per, t_last), lA, gA);
        load_epi(t, eC);   // (after the halo, as in the loop: the loop head's vmcnt waits then
                           // count the same ops on entry and on the back edge, not vmcnt(0))
      }
    }
    __syncthreads();   // weights + first halos
    int dsel = 0;   // (D3) the dY buffer of tile t
    auto step = [&](u32x4 (&lc)[D_ITD], u32x4 (&gc)[D_ITD], const u32x2 (&ec)[MT][NE], u32x2 (&en)[MT][NE],
                    int cur) -> bool {
      const int t1 = t + per;
      if constexpr (DDMA) {   // tile t + 2 per's dY halo DMA'd after this tile's epilogue
        constexpr int NST = W16 ? NTL : MT * NTL;   // epilogue loads = dX stores per lane
        load_epi(min(t1, t_last), en);
        dgrad_tile(t, ec, dsel * Cfg::D_BYTES);
        issue_d(min(t + 2 * per, t_last), (dsel == 0 ? 2 : dsel - 1) * Cfg::D_BYTES);
        dw_wait_vm<2 * NST + Cfg::D_PIECES / 4>();   // tile t1's DMA (issued one step ago) done
        __syncthreads();
        dsel = dsel == 2 ? 0 : dsel + 1;
        t = t1;
        return t < t_hi;
      }
#ifdef DW_STAMPS
      const unsigned long long s0 = DW_NOW();
#endif
      store(lc, gc, half == 0 && t1 < t_hi, (cur ^ 1) * Cfg::D_BYTES);   // (past the range: a re-read of the last tile)
#ifdef DW_STAMPS
      const unsigned long long s1 = DW_NOW();
#endif
      load(min(t + 2 * per, t_last), lc, gc);
      load_epi(min(t1, t_last), en);
#ifdef DW_STAMPS
      const unsigned long long s2 = DW_NOW();
#endif
      dgrad_tile(t, ec, cur * Cfg::D_BYTES);   // MFMAs + dX stores
#ifdef DW_STAMPS
      const unsigned long long s4 = DW_NOW();
#endif
      __syncthreads();   // buffer cur consumed, buffer cur^1 written
#ifdef DW_STAMPS
      const unsigned long long s5 = DW_NOW();
      st[0] += s1 - s0; st[1] += s2 - s1; st[2] += st_mid - s2; st[3] += s4 - st_mid; st[4] += s5 - s4; st[6] += 1;
#endif
      t = t1;
      return t < t_hi;
    };
    if (t < t_hi)
      while (step(lA, gA, eC, eN, 0) && step(lA, gA, eN, eC, 1)) {}
    // the last step issued one more DMA (a re-read of the last tile): it must land before
    // the block's LDS is released (or, with partials, re-used below)
    if constexpr (DDMA) dw_wait_vm<0>();
    } else {
    if (t < t_hi) {
      load(t, lA, gA);
      store(lA, gA, half == 0, 0);
      load_epi(t, eC);
      load(min(t + per, t_last), lA, gA);
    }
    __syncthreads();   // weights + first halos
    auto step = [&](u32x4 (&lc)[D_ITD], u32x4 (&gc)[D_ITD], u32x4 (&ln)[D_ITD], u32x4 (&gn)[D_ITD],
                    const u32x2 (&ec)[MT][NE], u32x2 (&en)[MT][NE]) -> bool {
      const int t1 = t + per;
      load(min(t + 2 * per, t_last), ln, gn);
      load_epi(min(t1, t_last), en);
      dgrad_tile(t, ec, 0);   // MFMAs + dX stores
      __syncthreads();   // halos of t consumed
      store(lc, gc, half == 0 && t1 < t_hi, 0);   // unconditional (past the range: a re-read of the last tile)
      __syncthreads();   // halos of t1 visible
      t = t1;
      return t < t_hi;
    };
    if (t < t_hi)
      while (step(lA, gA, lB, gB, eC, eN) && step(lB, gB, lA, gA, eN, eC)) {}
    }

    // dalpha / dbias partials of this split into LDS (the loop ended with a barrier
    // that both roles passed, so the halo area is free); summed below
    if constexpr (GO) {   // (the weight panel is dead too: the finished layer's partials)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int m = 1; m < 16; m <<= 1) {   // over the 16 pixel columns r
            gsa[jn][e] += __shfl_xor(gsa[jn][e], m, 64);
            gsb[jn][e] += __shfl_xor(gsb[jn][e], m, 64);
          }
      if (r == 0) {
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gred[(rw * 2 + 0) * BN + jn * 16 + 4 * g + e] = gsa[jn][e];
            gred[(rw * 2 + 1) * BN + jn * 16 + 4 * g + e] = gsb[jn][e];
          }
      }
    }
    if (GT && wg.part) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        red[rt * VEC + k] = sa[k];
        red[RED_T * VEC + rt * VEC + k] = sb[k];
      }
    }
  } else {
    // ================= W waves: X halo, wgrad
    const int xc0 = wg.b_c0 + col0;
    const int xupp = (wg.b_pl && xc0 % wg.b_ps == 0 && XU % (wg.b_ps / VEC) == 0) ? (int)(wg.b_ps / VEC) : XU;
    // per unit: global offset and LDS offset (-1: padding unit; its halo pixel is
    // llds / XROW, so no third array)
    // (XREC: the two index arrays recomputed per use instead of held -- tried for the W
    // share of the widest shape, it spilled more)
    constexpr bool XREC = false;
    auto xunit = [&](int it, int& rel, int& ll) {
      const int u = rt + it * NR;
      const int pln = u / (HW_ * xupp), rem = u - pln * (HW_ * xupp);
      const bool ok = u < X_UNITS;
      const int hq = ok ? rem / xupp : 0, cu = ok ? pln * xupp + rem % xupp : 0;
      const int hy = hq / RS, hx = hq - hy * RS;
      rel = (hy * W + hx) * (int)wg.b_ps + rdn_coff32(xc0 + cu * VEC, (int)wg.b_ps, (int)wg.b_pl);
      ll = ok ? hq * XROW + cu * 16 : -1;
    };
    int lrel_[XREC ? 1 : X_IT], llds_[XREC ? 1 : X_IT];
    if constexpr (!XREC) {
#pragma unroll
      for (int it = 0; it < X_IT; ++it) xunit(it, lrel_[it], llds_[it]);
    }
    auto xrel = [&](int it) {
      if constexpr (XREC) {
        int rel, ll;
        xunit(it, rel, ll);
        return rel;
      } else {
        return lrel_[it];
      }
    };
    auto xlds = [&](int it) {
      if constexpr (XREC) {
        int rel, ll;
        xunit(it, rel, ll);
        return ll;
      } else {
        return llds_[it];
      }
    };
    auto load = [&](int tt, u32x4 (&lr)[X_IT]) {
      int oy, ox, on;
      origin(tt, oy, ox, on);
      const int64_t hpix0 = ((int64_t)on * H + (oy - 1)) * W + (ox - 1);
      const __amdgpu_buffer_rsrc_t rx = rdn_rsrc(XS + hpix0 * wg.b_ps);
#pragma unroll
      for (int it = 0; it < X_IT; ++it) {
        const int ll = xlds(it);
        lr[it] = rdn_ld16(rx, in_img(ll < 0 ? HW_ : ll / XROW, oy, ox), xrel(it) * 2);
      }
    };
    auto store = [&](const u32x4 (&lr)[X_IT], int xoff) {
#pragma unroll
      for (int it = 0; it < X_IT; ++it) {
        const int ll = xlds(it);
        *(u32x4*)(ll >= 0 ? xh + xoff + ll : dump + rt * 16) = lr[it];
      }
    };
    // (WSH) dY halo unit DN + rt: loaded, gated (the D waves' fast packed gate, or the
    // scalar one with the dalpha/dbias partials of a tile-interior unit) and stored to
    // the same LDS image as the D waves' units
    const int wdcu = rt % DU;
    int wlrel = 0, wgrel = 0, wllds = 0, whp = HW_;
    bool wint = false;
    float wsa[VEC], wsb[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      wsa[q] = 0.f;
      wsb[q] = 0.f;
    }
    if constexpr (WSH) {
      const int u = DN + rt;
      int hp = u < D_UNITS ? u / DU : HW_;
      if constexpr (BSPLIT) {   // halo-ring pixel bp: top row, bottom row, left column, right column
        const int bp = rt / DU;
        hp = rt >= D_UNITS - IU ? HW_
             : bp < RS         ? bp
             : bp < 2 * RS     ? (TH + 1) * RS + bp - RS
             : bp < 2 * RS + TH ? (bp - 2 * RS + 1) * RS
                                : (bp - 2 * RS - TH + 1) * RS + RS - 1;
      }
      const int hq = hp < HW_ ? hp : 0;
      const int hy = hq / RS, hx = hq - hy * RS;
      whp = hp;
      wlrel = (hy * W + hx) * (int)d.x_ps + rdn_coff32(d.x_c0 + wdcu * VEC, (int)d.x_ps, (int)d.x_pl);
      wgrel = (hy * W + hx) * (int)d.gate_ps + rdn_coff32(wdcu * VEC, (int)d.gate_ps, (int)d.gate_pl);
      wllds = hq * DROW + wdcu * 16;
      wint = hp < HW_ && hy >= 1 && hy <= TH && hx >= 1 && hx <= TW;
    }
    auto loadD = [&](int tt, u32x4& lr, u32x4& gr) {
      int oy, ox, on;
      origin(tt, oy, ox, on);
      const int64_t hpix0 = ((int64_t)on * H + (oy - 1)) * W + (ox - 1);
      const bool ok = in_img(whp, oy, ox);
      lr = rdn_ld16(rdn_rsrc(DY + hpix0 * d.x_ps), ok, wlrel * 2);
      if constexpr (GT) gr = rdn_ld16(rdn_rsrc(PR + hpix0 * d.gate_ps), ok, wgrel * 2);
      else gr = u32x4{0u, 0u, 0u, 0u};
    };
    auto storeD = [&](const u32x4& lr, const u32x4& gr, bool live, int doff) {
      unsigned char* const dst = whp < HW_ ? dyh + doff + wllds : dump + rt * 16;
      if constexpr (!GT) {
        *(u32x4*)dst = lr;
      } else {
        const f32x4 a0 = *(const f32x4*)(alds + wdcu * VEC), a1 = *(const f32x4*)(alds + wdcu * VEC + 4);
        if (BSPLIT || !live) {   // (block-uniform) the packed gate, no partials
          u32x4 o;
          o[0] = rdn_gate2(lr[0], gr[0], a0[0], a0[1]);
          o[1] = rdn_gate2(lr[1], gr[1], a0[2], a0[3]);
          o[2] = rdn_gate2(lr[2], gr[2], a1[0], a1[1]);
          o[3] = rdn_gate2(lr[3], gr[3], a1[2], a1[3]);
          *(u32x4*)dst = o;
          return;
        }
        float dy[VEC], pr[VEC];
        Unit16<bf16>::unpack(lr, dy);
        Unit16<bf16>::unpack(gr, pr);
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const bool pos = pr[q] > 0.f;
          if (wint && !pos) wsa[q] += pr[q] * dy[q];
          dy[q] = pos ? dy[q] : (q < 4 ? a0[q] : a1[q - 4]) * dy[q];
          if (wint) wsb[q] += dy[q];
        }
        *(u32x4*)dst = Unit16<bf16>::pack(dy);
      }
    };
    // lane (g, q = r>>2, pp = r&3) supplies pixels {4g+q, 16+4g+q} of each 32-pixel
    // k-step (tile rows 2ks, 2ks+1) and channels / columns 4pp..4pp+3
    const int q4 = r >> 2, pp = r & 3;
    const unsigned char* const pwa = dyh + (RS + 4 * g + q4 + 1) * DROW + (DDMA ? 0 : 4 * pp * 2);   // interior (0, 4g+q)
    // in-row byte offset of m-tile i's channels 16 i + 4 pp .. +3 (DDMA: the unit of halo
    // column 4g+q+1 swizzled)
    int wsw[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i)
      wsw[i] = DDMA ? (((2 * i + (pp >> 1)) ^ ((4 * g + q4 + 1) & 7)) * 16 + (pp & 1) * 8) : i * 32;
    const unsigned char* const pwb = xh + (4 * g + q4) * XROW;
    auto boff = [&](int j) {   // column offset of n-tile rw + 4 j (recomputed: registers)
      const int nt = rw + 4 * j;
      const int c = nt < NT_ALL ? nt * 16 + 4 * pp : 0;
      const int tp = c / BN, ci = c - (c / BN) * BN;
      return ((tp / 3) * RS + tp % 3) * XROW + ci * 2;
    };
    f32x4 accW[MTW][NTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) accW[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // (k-step, n-tile) steps in one software pipeline: the B fragments of step s + PD
    // are read before step s's MFMAs, the A fragments of k-step ks + 1 at the start of
    // ks (the plain per-k-step form waited on each fragment right after reading it:
    // with MTW = 1-2 MFMAs per fragment the LDS latency was exposed at every step)
    auto wgrad_tile = [&](int xoff, int doff) {
      constexpr int PD = DW_WPIPE, NQ = PD + 1, KS = TH / 2, NS = KS * NTW;
      auto rdA = [&](int ks, bf16x8 (&a)[MTW]) {
#pragma unroll
        for (int i = 0; i < MTW; ++i) {
          const i16x4 lo =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, pwa + doff + (2 * ks) * RS * DROW + wsw[i]));
          const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              RDN_LDS_PTR(i16x4, pwa + doff + (2 * ks + 1) * RS * DROW + wsw[i]));
          a[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      };
      auto rdB = [&](int st) {   // (an n-tile past NT_ALL reads column 0: uniform, unused)
        const unsigned char* b = pwb + xoff + boff(st % NTW) + (2 * (st / NTW)) * RS * XROW;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b + RS * XROW));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      };
      bf16x8 af[2][MTW], bq[NQ];
      rdA(0, af[0]);
#pragma unroll
      for (int p = 0; p < PD && p < NS; ++p) bq[p] = rdB(p);
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        const int ks = st / NTW, j = st % NTW;
        if (j == 0 && ks + 1 < KS) rdA(ks + 1, af[(ks + 1) & 1]);
        if (st + PD < NS) bq[(st + PD) % NQ] = rdB(st + PD);
        if (rw + 4 * j < NT_ALL) {   // wave-uniform
#pragma unroll
          for (int i = 0; i < MTW; ++i)
            accW[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bq[st % NQ], accW[i][j], 0, 0, 0);
        }
      }
    };
    if constexpr (Cfg::SB) {
    // the D waves' schedule (one barrier per tile): step k computes tile t from X
    // buffer k&1 (and the dY halo buffer k&1) while tile t + per, issued one step
    // earlier, goes to buffer (k+1)&1.  One register set for every shape (two, for
    // the shapes whose budget held them, spilled once both parities were unrolled)
    // and a run-time parity (unrolled, the two copies spilled the 64 / 80-column ones)
    {
      u32x4 lA[X_IT], dl = {0u, 0u, 0u, 0u}, dg = {0u, 0u, 0u, 0u};
      if (t < t_hi) {
        load(t, lA);
        if constexpr (WSH) loadD(t, dl, dg);
        store(lA, 0);
        if constexpr (WSH) storeD(dl, dg, half == 0, 0);
        load(min(t + per, t_last), lA);
        if constexpr (WSH) loadD(min(t + per, t_last), dl, dg);
      }
      __syncthreads();   // weights + first halos
      for (int k = 0; t < t_hi; ++k) {
        const int cur = k & 1;
#ifdef DW_STAMPS
        const unsigned long long s0 = DW_NOW();
#endif
        store(lA, (cur ^ 1) * Cfg::X_BYTES);   // tile t + per (a re-read past the range)
        if constexpr (WSH) storeD(dl, dg, half == 0 && t + per < t_hi, (cur ^ 1) * Cfg::D_BYTES);
#ifdef DW_STAMPS
        const unsigned long long s1 = DW_NOW();
#endif
        load(min(t + 2 * per, t_last), lA);
        if constexpr (WSH) loadD(min(t + 2 * per, t_last), dl, dg);
#ifdef DW_STAMPS
        const unsigned long long s2 = DW_NOW();
#endif
        wgrad_tile(cur * Cfg::X_BYTES, (Cfg::D3 ? k % 3 : cur) * Cfg::D_BYTES);
#ifdef DW_STAMPS
        const unsigned long long s3 = DW_NOW();
#endif
        __syncthreads();   // buffers cur consumed, buffers cur^1 written
#ifdef DW_STAMPS
        const unsigned long long s4 = DW_NOW();
        st[0] += s1 - s0; st[1] += s2 - s1; st[2] += s3 - s2; st[4] += s4 - s3; st[6] += 1;
#endif
        t += per;
      }
    }
    } else {
    if constexpr (DW2) {   // two tiles in flight: register sets alternate
      u32x4 lA[X_IT], lB[X_IT];
      if (t < t_hi) {
        load(t, lA);
        store(lA, 0);
        load(min(t + per, t_last), lA);
      }
      __syncthreads();   // weights + first halos
      auto step = [&](u32x4 (&lc)[X_IT], u32x4 (&ln)[X_IT]) -> bool {
        load(min(t + 2 * per, t_last), ln);
        wgrad_tile(0, 0);
        __syncthreads();   // halos of t consumed
        store(lc, 0);
        __syncthreads();   // halos of t1 visible
        t += per;
        return t < t_hi;
      };
      if (t < t_hi)
        while (step(lA, lB) && step(lB, lA)) {}
    } else if constexpr (Cfg::XB == 2) {
      // one register set, two X halo buffers: at the top of step k the set holds tile
      // k+1 (issued a whole step earlier); it goes to buffer (k+1)&1 -- free since
      // step k-1's MFMAs -- and takes tile k+2 while tile k computes from buffer k&1
      u32x4 lA[X_IT];
      if (t < t_hi) {
        load(t, lA);
        store(lA, 0);
        load(min(t + per, t_last), lA);
      }
      __syncthreads();   // weights + first halos
      int k = 0;
      while (t < t_hi) {
        store(lA, ((k + 1) & 1) * Cfg::X_BYTES);   // tile t + per (a re-read past the range)
        load(min(t + 2 * per, t_last), lA);
        wgrad_tile((k & 1) * Cfg::X_BYTES, 0);
        __syncthreads();   // halos of t consumed; X of t + per visible
        __syncthreads();   // (the D waves' dY halo of t + per)
        t += per;
        ++k;
      }
    } else {   // one tile of X in flight (96 columns: neither budget holds two)
      u32x4 lA[X_IT];
      if (t < t_hi) {
        load(t, lA);
        store(lA, 0);
      }
      __syncthreads();   // weights + first halos
      while (t < t_hi) {
        load(min(t + per, t_last), lA);
        wgrad_tile(0, 0);
        __syncthreads();   // halos of t consumed
        store(lA, 0);
        __syncthreads();   // halos of t1 visible
        t += per;
      }
    }

    }

    // this block's split of the weight gradient (zero slab for a block without tiles);
    // halves: the slab holds this half's 9 x BN columns only
    const int ncolw = NH > 1 ? BN : wg.ndim;
    const int ncol_all = 9 * ncolw;
    float* __restrict__ ws = wg.ws + (int64_t)slab * wg.mdim * ncol_all;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int nt = rw + 4 * j;
      if (nt >= NT_ALL) continue;
      const int c = nt * 16 + r;
      const int tp = c / BN, ci = c - tp * BN;
      const int col = tp * ncolw + ci;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = i * 16 + g * 4 + e;
          if (m < wg.mdim) ws[(int64_t)m * ncol_all + col] = accW[i][j][e];
        }
    }
    if constexpr (WSH) {   // (the loop's last barrier freed the halo area, as for the D waves)
      if (GT && wg.part) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          red[(NR + rt) * VEC + k] = wsa[k];
          red[RED_T * VEC + (NR + rt) * VEC + k] = wsb[k];
        }
      }
    }
  }

  // dalpha / dbias partials of this split, fixed order.  Both roles arrive at this
  // ONE barrier (each role's loop passes the same number of barriers per tile), so
  // no barrier is ever role-divergent.
  if (GT && wg.part) {
    __syncthreads();
    if (dwave && rt < CK) {
      constexpr int DUC = CK / VEC;
      const int cg = rt / VEC, k = rt % VEC;
      float a = 0.f, b = 0.f;
      for (int rr = 0; rr < RED_T / DUC; ++rr) {   // D threads, then (WSH) W threads
        a += red[(rr * DUC + cg) * VEC + k];
        b += red[RED_T * VEC + (rr * DUC + cg) * VEC + k];
      }
      if (rt < wg.mdim) {
        wg.part[((int64_t)slab * 2 + 0) * wg.mdim + rt] = a;   // (zero rows in half 1)
        wg.part[((int64_t)slab * 2 + 1) * wg.mdim + rt] = b;
      }
    }
    if constexpr (GO) {   // the finished layer's row `slab`: this half's columns, zeros elsewhere
      if (dwave) {
        const int gcn = d.ncols - d.gout_c0;
        float* const prt = d.gout_part + (int64_t)slab * 2 * gcn;
        for (int j = rt; j < gcn; j += NR) {
          const int cl = d.gout_c0 + j - col0;
          float a = 0.f, b = 0.f;
          if (cl >= 0 && cl < BN) {
            a = (gred[0 * BN + cl] + gred[2 * BN + cl]) + (gred[4 * BN + cl] + gred[6 * BN + cl]);
            b = (gred[1 * BN + cl] + gred[3 * BN + cl]) + (gred[5 * BN + cl] + gred[7 * BN + cl]);
          }
          prt[j] = a;
          prt[gcn + j] = b;
        }
      }
    }
  }
#ifdef DW_STAMPS
  {   // (a per-lane vector store: lane q writes phase q)
    unsigned long long v = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) v = lane == q ? st[q] : v;
    if (lane < 8) g_dw_st[((int64_t)blockIdx.x * 8 + wave) * 8 + lane] = v;
  }
#endif
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
// multiple of 8: the XCD tile ranges), at most the tiles of an XCD's share (per
// column half: nh halves take nh blocks per XCD slot)
int dw_grid(int ntiles, int nh = 1) {
  const int per_xcd = (ntiles + 7) / 8;
  int slots = device_cus() / (8 * nh);
  if (slots > per_xcd) slots = per_xcd;
  if (slots < 1) slots = 1;
  return 8 * nh * slots;
}

// column halves for this pair: 2 for the 96 / 128-input-channel convs with 32 dY
// channels (level-1 conv_1 / conv_2), else 1
// (RDN_DW_HALVES=0: only the single-tile shapes, for A/B)
bool dw_halves_enabled() {
  static const bool on = [] {
    const char* e = getenv("RDN_DW_HALVES");
    return !(e && e[0] == '0');
  }();
  return on;
}
int dw_nh(const rdn_conv_desc* d) {
  if (!dw_halves_enabled()) return 1;
  if (d->cin == 32 && (d->ncols == 96 || d->ncols == 128)) return 2;
  static const bool h5 = [] {   // (RDN_DW_H5=0: the level-1 conv_3 on the separate kernels, for A/B)
    const char* e = getenv("RDN_DW_H5");
    return !(e && e[0] == '0');
  }();
  if (h5 && d->cin == 64 && d->ncols == 160) return 5;   // level-1 conv_3: five 32-channel parts
  return 1;
}

// gate-out (d->gout) on this pair: the instantiated shapes (up_0.conv: 96 columns in
// halves; the level-1 conv_0: 64 columns), whole 4-channel units, 8-byte aligned
// operands, 32-bit per-tile offsets
bool dw_gout_ok(const rdn_conv_desc* d, const rdn_wgrad_desc* wg) {
  const int nh = dw_nh(d);
  if (d->cin != 32 || !((d->ncols == 96 && nh == 2) || (d->ncols == 64 && nh == 1))) return false;
  if (!d->gout_pre || !d->gout_alpha || !d->gout_part || !wg->part || (d->flags & RDN_EPI_RESID)) return false;
  if (d->gout_c0 < 0 || d->gout_c0 >= d->ncols || d->gout_c0 % 4 || d->gout_ps % 4 || d->gout_pre_ps % 4) return false;
  if (d->gout_ps < d->ncols - d->gout_c0 || d->gout_pre_ps < d->ncols - d->gout_c0) return false;
  if (((uintptr_t)d->gout & 7) || ((uintptr_t)d->gout_pre & 7) || ((uintptr_t)d->gout_part & 3)) return false;
  return (int64_t)TH * d->w * d->gout_ps < (1ll << 30) && (int64_t)TH * d->w * d->gout_pre_ps < (1ll << 30);
}

// the pair this kernel serves (else 1 = run the separate dgrad / wgrad launches)
bool dw_serves(const rdn_conv_desc* d, const rdn_wgrad_desc* wg) {
  if (!dw_enabled() || !d || !wg) return false;
  if (d->dtype != RDN_BF16 || wg->dtype != RDN_BF16 || d->gather != RDN_G_CONV3 || wg->gather != RDN_G_CONV3) return false;
  if (d->bn || d->bm) return false;
  // gated (the loaders apply the PReLU backward, dalpha/dbias partials in wg->part) or,
  // for the level-1 conv_3 only, pre-gated: the operand is the layer's dYpre (written
  // by a gate-out finisher or the PReLU-backward pass, which also count the partials)
  const bool gated = d->gate && wg->a_gate && d->gate_alpha;
  if (!gated && (d->gate || wg->a_gate || wg->part || !(d->cin == 64 && d->ncols == 160))) return false;
  if (d->gout && !dw_gout_ok(d, wg)) return false;
  if (d->flags & ~(RDN_EPI_RESID | RDN_EPI_ACCUM | (d->gout ? RDN_EPI_GOUT_KEEP : 0))) return false;
  if ((d->flags & RDN_EPI_RESID) && (d->flags & RDN_EPI_ACCUM)) return false;
  if (d->h % TH || d->w % TW || d->n != wg->n || d->h != wg->h || d->w != wg->w) return false;
  const int nh = dw_nh(d);
  if (d->cin != 16 && d->cin != 32 && !(d->cin == 64 && nh == 5)) return false;
  if (d->ncols != d->cout || d->ncols % 16 || d->ncols < 32 || d->ncols / nh > 80 || wg->ndim != d->ncols) return false;
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

template <int BN, int CK, int NH = 1, bool GO = false, bool GT = true>
int launch_dw(const rdn_conv_desc* d, const rdn_wgrad_desc* wg, hipStream_t st) {
  if constexpr (!DwCfg<BN, CK, GO, !GT && CK == 64 && !GO>::FITS) {
    return 1;
  } else {
    const int tiles_x = d->w / TW, tiles_y = d->h / TH;
    const int ntiles = d->n * tiles_x * tiles_y;
    const int grid = dw_grid(ntiles, NH);
    if (!GT) RDN_PROBE("conv3_dw_kernel<bf16,%d,%d,h%d,pregated>", BN, CK, NH);
    if (NH > 1) RDN_PROBE("conv3_dw_kernel<bf16,%d,%d,h%d%s>", BN, CK, NH, GO ? ",go" : "");
    RDN_PROBE("conv3_dw_kernel<bf16,%d,%d%s>", BN, CK, GO ? ",go" : "");
    if (wg->splits != grid) {
      rdn_set_error("rdn_conv_dgrad_wgrad: wgrad splits %d != %d (rdn_conv_dgrad_wgrad_splits)", wg->splits, grid);
      return RDN_E_ARG;
    }
    if (!wg->ws) { rdn_set_error("rdn_conv_dgrad_wgrad: null workspace"); return RDN_E_ARG; }
    hipLaunchKernelGGL((conv3_dw_kernel<BN, CK, NH, GO, GT>), dim3((unsigned)grid), dim3(NT), 0, st, *d, *wg, tiles_x,
                       tiles_y, ntiles);
    return rdn_check_launch("rdn_conv_dgrad_wgrad");
  }
}

template <int CK>
int dw_bn(const rdn_conv_desc* d, const rdn_wgrad_desc* wg, hipStream_t st) {
  if constexpr (CK == 64) {   // (dw_serves: the level-1 conv_3, 160 input channels in five parts)
    if (!d->gout && dw_nh(d) == 5 && d->ncols == 160)
      return d->gate ? launch_dw<32, 64, 5>(d, wg, st) : launch_dw<32, 64, 5, false, false>(d, wg, st);
    return 1;
  } else {
  if (d->gout) {   // (dw_gout_ok: these two shapes only)
    if constexpr (CK == 32) {
      if (d->ncols == 96) return launch_dw<48, 32, 2, true>(d, wg, st);
      if (d->ncols == 64) return launch_dw<64, 32, 1, true>(d, wg, st);
    }
    return 1;
  }
  if constexpr (CK == 32) {
    if (dw_nh(d) == 2) {
      switch (d->ncols) {
        case 96: return launch_dw<48, 32, 2>(d, wg, st);
        case 128: return launch_dw<64, 32, 2>(d, wg, st);
      }
      return 1;
    }
  }
  switch (d->ncols) {
    case 32: return launch_dw<32, CK>(d, wg, st);
    case 48: return launch_dw<48, CK>(d, wg, st);
    case 64: return launch_dw<64, CK>(d, wg, st);
    case 80: return launch_dw<80, CK>(d, wg, st);
  }
  return 1;
  }
}

int dw_dispatch(const rdn_conv_desc* d, const rdn_wgrad_desc* wg, hipStream_t st) {
  if (!dw_serves(d, wg)) return 1;
  return d->cin == 64 ? dw_bn<64>(d, wg, st) : d->cin == 32 ? dw_bn<32>(d, wg, st) : dw_bn<16>(d, wg, st);
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
  return dw_grid(dgrad->n * (dgrad->h / TH) * (dgrad->w / TW), dw_nh(dgrad));
}

// input channels per weight-gradient slab (= wgrad->ndim, or ndim / 2 with column
// halves: the slabs of half h are [h*splits/2, (h+1)*splits/2)), 0 if not served
extern "C" int rdn_conv_dgrad_wgrad_cols(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad) {
  if (!rdn_conv_dgrad_wgrad_splits(dgrad, wgrad)) return 0;
  return dgrad->ncols / dw_nh(dgrad);
}

// partial rows the gate-out epilogue writes for the finished layer (one per block of
// the persistent grid = the split count), 0 if this pair with its d->gout is not served
extern "C" int rdn_conv_dgrad_wgrad_gate_rows(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad) {
  if (!dgrad || !wgrad || !dgrad->gout) return 0;
  return rdn_conv_dgrad_wgrad_splits(dgrad, wgrad);
}

#ifdef DW_STAMPS
extern "C" int rdn_dw_stamps(unsigned long long* host, int32_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dw_st), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

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
