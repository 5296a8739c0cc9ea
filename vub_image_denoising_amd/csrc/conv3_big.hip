// 3x3 / pad 1 / stride 1 convolution as a persistent implicit GEMM on large tiles
// (gfx950, bf16 MFMA, LDS-DMA staging): the MFMA-heavy convolutions of levels 1-3
// in forward (Unet_model.py:72-89 dense convs, :35-43 up convs) and their input
// gradients (the same conv over dYpre with rotated, transposed weights).
//
// Why: conv3_halo (4 waves, 8 x 16 pixels x <= 128 columns) re-streams the weights
// from L2 for every 128 pixels and meets a barrier every 16-32 MFMAs per wave; at
// levels 2/3 it ran at 0.28-0.36 of the MFMA peak.  A first large-tile version of
// this kernel (one 16 x 16-pixel tile per block, register-staged, r03) showed what
// else limits: a level-2 grid is ONE round of blocks over the CUs, so every block
// loads its first halo, multiplies and writes its outputs in lock step with all
// the others, and the only variant that beat conv3_halo ran two blocks per CU.
// Here:
//
// * block = 512 threads (8 waves), one per CU, PERSISTENT over work items (a 16 x 16
//   pixel tile x BN output columns): the next item's first halo and weight stage
//   are in flight during the current item's last stages, and the epilogue goes
//   from the accumulators straight to global memory (buffer stores, no LDS tile,
//   no barrier), so its stores drain while the next item multiplies;
// * every weight byte staged in LDS feeds 256 pixels; each wave owns a 64 x 64
//   (64 x 32) accumulator tile: 128 B/clk/CU of LDS fragment reads at the MFMA
//   rate, half the LDS bandwidth;
// * everything reaches LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging):
//   the input halo [18 x 18][CK] of a channel chunk (double buffered, loaded ONCE
//   for all 9 taps, one chunk ahead) and the weights (one LDS stage = two 64-deep
//   K stages, double buffered, one stage ahead); each wave waits for its own DMAs
//   with a counted vmcnt and a raw barrier publishes them.  A DMA wave-instruction
//   writes 1 KB linearly, so the LDS images are dense and bank conflicts of the
//   ds_read_b128 fragment reads are removed by XOR-swizzling 16-byte units on the
//   SOURCE side (checked exhaustively for the fragment patterns, every tap shift);
// * MFMA operands are swapped (A = weights, B = pixels): a lane holds four
//   consecutive output channels of one pixel -- the 8-byte epilogue unit.
//
// Packed weights as for conv3_halo (rdn_pack_weights with ck > 0):
//   P[n][chunk*KC + tap*CK + ci],  KC = roundup(9*CK, 64).
#include "conv3_tile.h"

#include <cstdlib>

namespace {

__device__ __attribute__((aligned(64))) unsigned int g_big_zero[16];

// Round 5: pairs of pixel rows are exchanged between lane rows g, g^1 (v_permlane16_swap)
// so the epilogue moves 16-byte units (8 channels of one pixel) instead of 8-byte ones:
// half the epilogue memory instructions (as conv3_dw's dX epilogue), except gate-out.
// Round 4: the next k-step's fragments are read before the current MFMAs (two fragment
// sets live; bit-identical; B16 +0.6 %, B32 +0.5 %, profiles/r04_v5_big_pf_gate_out_ab.txt).

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// One LDS-DMA wave-instruction: 16 B per lane from `src` to LDS byte dst + lane*16
// (dst wave-uniform, in M0).  Inline asm, so that the compiler does not treat the
// LDS as pending on the VM counter (with the builtin it waits vmcnt(0) before every
// ds_read of the array); the counted waits in the loop are the ordering.
__device__ __forceinline__ void glds16(const void* src, unsigned dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const unsigned char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

constexpr int TWB = 16;
constexpr int RS = TWB + 2;        // halo pixels per halo row
constexpr int LDS_CAP = 160 * 1024;
constexpr int COL_MAX = 640;       // bias / PReLU-slope table in LDS

// epilogue modes (compile-time): forward = bias + PReLU-input store + PReLU
// (+ residual); input gradient = plain (+ accumulate | + residual)
enum { EP_FWD = 0, EP_FWD_RES = 1, EP_PLAIN = 2, EP_ACC = 3, EP_RES = 4 };

// halo image swizzle: physical 16-B unit of logical unit u at halo column x
template <int CK>
__device__ __forceinline__ int hswz(int u, int x) {
  return CK == 64 ? (u ^ (x & 7)) : (u ^ ((x >> 1) & 3));
}

// NW waves per block: 8 = one block per CU (the LDS-heavy shapes); 4 = a 4-wave block
// with half the LDS budget, two blocks per CU (see conv3_big_kernel's note on BIG_NW4)
template <int TH, int BN, int WM, int CK, int NW = 8>
struct PtCfg {
  static constexpr int NTB = 64 * NW;
  static constexpr int BPC = NW == 8 ? 1 : 2;                  // blocks per CU
  static constexpr int BM = TH * TWB;
  static constexpr int HWP = (TH + 2) * RS;                    // halo pixels
  static constexpr int RB = CK * 2;                            // bytes per halo pixel
  static constexpr int H_PIECES = (HWP * RB + 1023) / 1024;    // 1-KB DMA pieces per halo
  static constexpr int HALO_BYTES = H_PIECES * 1024;
  static constexpr int KC = (9 * CK + 63) / 64 * 64;           // packed K per chunk
  static constexpr int SPC = KC / 64;                           // 64-deep K stages per chunk
  static constexpr int SS = (SPC + 1) / 2;                      // LDS stages (pairs) per chunk
  static constexpr int RW = 256;                                // LDS weight row: 2 x 128 B
  static constexpr int W_BYTES = BN * RW;
  static constexpr int W_PIECES = W_BYTES / 1024;
  static constexpr int W_PW = (W_PIECES + NW - 1) / NW;         // weight pieces per wave per stage (max)
  static constexpr int TAB = 2 * COL_MAX * 4;
  static constexpr int LDS = 2 * HALO_BYTES + 2 * W_BYTES + TAB;
  static constexpr int WN = NW / WM;
  static constexpr int WTM = BM / WM, WTN = BN / WN;            // wave tile (pixels x columns)
  static constexpr int MT = WTM / 16, NTL = WTN / 16;
  static constexpr bool OK = BPC * LDS <= LDS_CAP && MT >= 1 && NTL >= 1 && WTM % 16 == 0 && WTN % 16 == 0 &&
                             (CK == 32 || CK == 64) && WM * WN == NW && (NW == 8 || NW == 4);
};

template <int NLO, int NHI, int SPLIT>
__device__ __forceinline__ void wait_split(int wave) {   // vmcnt(wave < SPLIT ? NHI : NLO)
  if (wave < SPLIT) wait_vm<NHI>();
  else wait_vm<NLO>();
}

// launch bounds: 512 threads = 8 waves = two per SIMD, i.e. one block per CU (the LDS
// budget allows no more); the second argument is waves per SIMD (EU), so the register
// cap it implies is 256 VGPRs per lane (the most a 512-thread block can have; a bound of
// 1 would not raise it).  Round-4 end, -Rpass-analysis=kernel-resource-usage
// (profiles/r04_final_conv3_big_resources.txt): 139-251 VGPRs, no scratch, except the
// 128-column CK=64 items at 253-255 VGPRs, four of which (EP=1; EP=2..4 with GO) spill
// 20-36 B/lane -- the next register cut is there (a 128-column wave tile split)
//
// BIG_NW4 (round 5): at one 8-wave block per CU every wave reaches the same phase at
// the same time -- the LDS-DMA issue after a barrier, the stage barriers, the item's
// epilogue -- and the MFMA pipe idles through all of them.  Diagnostic builds on the
// level-1 conv_3 forward (160 -> 64, B16, scripts/kbench.py, profiles/r05_bigdiag_kbench.txt):
// 65.1 us as built; 44.6 without the in-loop DMAs, 51.9 without the epilogue, 53.0
// without the stage waits + barriers, 25.0 with the MFMAs alone.  The 4-wave variant
// (64 x 64 wave tiles) runs two independent blocks per CU, so one block's DMA issue,
// barrier skew and epilogue overlap the other's MFMAs
template <int TH, int BN, int WM, int CK, int EP, bool GO, int NW = 8>
__global__ __launch_bounds__(64 * NW, 2) void conv3_big_kernel(rdn_conv_desc d, int tiles_x, int tiles_y, int nitems) {
  using Cfg = PtCfg<TH, BN, WM, CK, NW>;
  constexpr int NTB = Cfg::NTB;
  constexpr int RB = Cfg::RB, RW = Cfg::RW, SPC = Cfg::SPC, SS = Cfg::SS;
  constexpr int WTN = Cfg::WTN, MT = Cfg::MT, NTL = Cfg::NTL, W_PW = Cfg::W_PW, HP = Cfg::H_PIECES;
  constexpr bool FWD = EP == EP_FWD || EP == EP_FWD_RES;
  constexpr bool RES = EP == EP_FWD_RES || EP == EP_RES;
  constexpr bool ACC = EP == EP_ACC;
  constexpr bool GOK = GO && !FWD;   // gate-out epilogue (input gradients only)
  constexpr bool W16 = !GOK && MT % 2 == 0;   // (launch_pt checks the 8-channel alignment)
  static_assert(Cfg::OK, "conv3_big geometry");

  __shared__ __attribute__((aligned(1024))) unsigned char lds[Cfg::LDS];
  unsigned char* const halo = lds;                               // two halo images
  unsigned char* const wst = lds + 2 * Cfg::HALO_BYTES;          // two weight stages
  float* const tab = (float*)(wst + 2 * Cfg::W_BYTES);           // [0, COL_MAX): bias, then slopes

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int r = lane & 15, g = lane >> 4;
  const int ncb = d.ncols / BN;
  const int H = d.h, W = d.w;
  const int nch = d.cin / CK;

  // this block's items: its XCD's contiguous share, strided by the XCD's block count
  // (consecutive items = the column blocks of one pixel tile: one halo, one L2)
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7;
  const int it_lo = (int)((int64_t)nitems * xcd / 8), it_hi = (int)((int64_t)nitems * (xcd + 1) / 8);
  int item = it_lo + (blockIdx.x >> 3);

  const bool spre = (d.flags & RDN_EPI_STORE_PRE) != 0;   // (forward-only: no PReLU input kept)
  if constexpr (FWD) {
    for (int c = tid; c < d.ncols; c += NTB) {
      tab[c] = d.bias[c];
      tab[COL_MAX + c] = d.alpha[c];
    }
  }
  if constexpr (GOK) {   // slopes of the gated layer (columns gout_c0.. of this conv)
    for (int c = tid; c < d.ncols - d.gout_c0; c += NTB) tab[COL_MAX + c] = d.gout_alpha[c];
  }

  struct Geo { int nimg, y0, x0, n0; };
  auto geo = [&](int itm) {
    Geo q;
    const int cb = itm % ncb;
    int t = itm / ncb;
    const int tx = t % tiles_x;
    t /= tiles_x;
    q.y0 = (t % tiles_y) * TH;
    q.x0 = tx * TWB;
    q.nimg = t / tiles_y;
    q.n0 = cb * BN;
    return q;
  };

  // ---- halo DMA of chunk c of item q into halo buffer hb: piece pc (wave w takes
  // pieces w, w + 8, ...) covers image bytes pc*1024 + lane*16 -> pixel hp, physical
  // unit pu holding logical unit hswz(pu, hx); out-of-image pixels read zeros
  auto issue_h = [&](const Geo& q, int c, int hb) {
    const unsigned dst = lds_addr(halo) + hb * Cfg::HALO_BYTES;
    const bf16* const xb = (const bf16*)d.x + (((int64_t)q.nimg * H + (q.y0 - 1)) * W + (q.x0 - 1)) * d.x_ps;
#pragma unroll
    for (int k = 0; k < (HP + NW - 1) / NW; ++k) {
      const int pc = wave + NW * k;
      if (pc >= HP) break;   // wave-uniform
      const int off = pc * 1024 + lane * 16;
      const int hp = off / RB, pu = (off % RB) / 16;
      const int hy = hp / RS, hx = hp - (hp / RS) * RS;
      const int u = hswz<CK>(pu, hx);
      const bool ok =
          hp < Cfg::HWP && (unsigned)(q.y0 - 1 + hy) < (unsigned)H && (unsigned)(q.x0 - 1 + hx) < (unsigned)W;
      const void* src = ok ? (const void*)(xb + (int64_t)(hy * W + hx) * d.x_ps +
                                           rdn_coff32(d.x_c0 + c * CK + u * 8, (int)d.x_ps, (int)d.x_pl))
                           : (const void*)g_big_zero;
      glds16(src, dst + pc * 1024);
    }
  };
  // ---- weight DMA: LDS stage (c, jj) holds K stages 2jj, 2jj+1 of chunk c (16 units
  // = 256 B of every output column n0..n0+BN); physical unit p of row n holds logical
  // unit p ^ (n & 15); the odd stage past a chunk's K loads zeros
  auto issue_w = [&](int n0, int c, int jj, int wb) {
    const unsigned dst = lds_addr(wst) + wb * Cfg::W_BYTES;
#pragma unroll
    for (int k = 0; k < W_PW; ++k) {
      const int pc = wave + NW * k;                    // piece: rows 4 pc .. 4 pc + 3
      if (pc >= Cfg::W_PIECES) break;                  // wave-uniform
      const int row = 4 * pc + (lane >> 4);
      const int u = (lane & 15) ^ (row & 15);
      const bool ok = 2 * jj + 1 < SPC || u < 8;
      const void* src = ok ? (const void*)((const bf16*)d.wp + (int64_t)(n0 + row) * d.kp + c * Cfg::KC + jj * 128 +
                                           u * 8)
                           : (const void*)g_big_zero;
      glds16(src, dst + pc * 1024);
    }
  };

  // ---- fragment addresses: lane (r, g) reads pixel column r + dx of its tile rows
  // (k unit g of the k-step) and weight row r of its column block (unit g)
  int a_off[CK == 64 ? 6 : 3];   // [ks][dx]: byte offset of the lane's swizzled unit
#pragma unroll
  for (int ks = 0; ks < (CK == 64 ? 2 : 1); ++ks)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) a_off[ks * 3 + dx] = (r + dx) * RB + hswz<CK>(ks * 4 + g, r + dx) * 16;
  const int a_row0 = (wm * MT) * RS * RB;
  const int b_lane = (wn * WTN + r) * RW;
  int b_off[4];   // per (K-stage half, k-step): swizzled unit of this lane's weight row
#pragma unroll
  for (int hk = 0; hk < 4; ++hk) b_off[hk] = ((hk * 4 + g) ^ r) * 16;

  f32x4 acc[MT][NTL];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // LDS stage jj of a chunk (K stages 2jj, 2jj+1) from halo image ph, weights pbs, as a
  // pipeline over its (up to) four 32-deep k-steps: the fragments of k-step q + 1 are
  // read before the MFMAs of q (two fragment sets live; same MFMA order: bit-identical)
  auto compute_pf = [&](int jj, const unsigned char* ph, const unsigned char* pbs) {
    auto valid = [&](int q) { return 2 * jj + (q >> 1) < SPC && (2 * jj + (q >> 1)) * 64 + (q & 1) * 32 < 9 * CK; };
    u32x4 af[2][MT], bfr[2][NTL];
    auto rd = [&](int q, int buf) {
#ifdef BIG_DIAG_NO_LDS   // diagnostic build (timing only): opaque fragments, no LDS reads
#pragma unroll
      for (int i = 0; i < MT; ++i) asm volatile("" : "=v"(af[buf][i]));
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) asm volatile("" : "=v"(bfr[buf][jn]));
      return;
#endif
      const int k0 = (2 * jj + (q >> 1)) * 64 + (q & 1) * 32;
      const int tap = k0 / CK, ksub = (k0 - tap * CK) / 32;
      const int dy = tap / 3, dx = tap % 3;
      const unsigned char* pa = ph + a_row0 + dy * RS * RB + a_off[ksub * 3 + dx];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[buf][i] = *(const u32x4*)(pa + i * RS * RB);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) bfr[buf][jn] = *(const u32x4*)(pbs + jn * 16 * RW + b_off[q]);
    };
    rd(0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!valid(q)) break;
      if (q + 1 < 4 && valid(q + 1)) rd(q + 1, (q + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);   // next k-step's reads issued before these MFMAs
#ifdef BIG_DIAG_NO_MFMA   // diagnostic build (timing only): fragments consumed without MFMAs
#pragma unroll
      for (int i = 0; i < MT; ++i) asm volatile("" ::"v"(af[q & 1][i]));
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) asm volatile("" ::"v"(bfr[q & 1][jn]));
      continue;
#endif
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)   // D[column][pixel]
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[q & 1][jn]),
                                                               __builtin_bit_cast(bf16x8, af[q & 1][i]), acc[i][jn], 0,
                                                               0, 0);
    }
  };
  // rolling form of the prefetch: the next k-step's weight fragments are read before
  // the MFMAs (double-buffered), each pixel fragment i of it right after the MFMAs that
  // read fragment i of this k-step (one buffer: MT x 4 fewer live registers; same MFMA
  // order, bit-identical)
  auto compute_roll = [&](int jj, const unsigned char* ph, const unsigned char* pbs) {
    auto valid = [&](int q) { return 2 * jj + (q >> 1) < SPC && (2 * jj + (q >> 1)) * 64 + (q & 1) * 32 < 9 * CK; };
    u32x4 af[MT], bfr[2][NTL];
    auto pa_of = [&](int q) {
      const int k0 = (2 * jj + (q >> 1)) * 64 + (q & 1) * 32;
      const int tap = k0 / CK, ksub = (k0 - tap * CK) / 32;
      const int dy = tap / 3, dx = tap % 3;
      return ph + a_row0 + dy * RS * RB + a_off[ksub * 3 + dx];
    };
    auto rdb = [&](int q, int buf) {
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) bfr[buf][jn] = *(const u32x4*)(pbs + jn * 16 * RW + b_off[q]);
    };
    {
      const unsigned char* pa = pa_of(0);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *(const u32x4*)(pa + i * RS * RB);
      rdb(0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!valid(q)) break;
      const bool nx = q + 1 < 4 && valid(q + 1);
      if (nx) rdb(q + 1, (q + 1) & 1);
      const unsigned char* pn = pa_of(nx ? q + 1 : q);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn)   // D[column][pixel]
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[q & 1][jn]),
                                                               __builtin_bit_cast(bf16x8, af[i]), acc[i][jn], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);   // (the reload may not move above the MFMAs reading af[i])
        if (nx) af[i] = *(const u32x4*)(pn + i * RS * RB);
      }
    }
  };
  // the same without the k-step prefetch: one fragment set live at a time
  auto compute_np = [&](int jj, const unsigned char* ph, const unsigned char* pbs) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * jj + h;
      if (j >= SPC) break;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int k0 = j * 64 + ks * 32;
        if (k0 >= 9 * CK) break;               // padded K: zero weights, skipped
        const int tap = k0 / CK, ksub = (k0 - tap * CK) / 32;
        const int dy = tap / 3, dx = tap % 3;
        const unsigned char* pa = ph + a_row0 + dy * RS * RB + a_off[ksub * 3 + dx];
        __builtin_amdgcn_sched_barrier(0);   // k-steps stay apart: one fragment set live at a time
        u32x4 af[MT], bfr[NTL];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = *(const u32x4*)(pa + i * RS * RB);
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) bfr[jn] = *(const u32x4*)(pbs + jn * 16 * RW + b_off[2 * h + ks]);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int jn = 0; jn < NTL; ++jn)   // D[column][pixel]
            acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[jn]),
                                                                 __builtin_bit_cast(bf16x8, af[i]), acc[i][jn], 0, 0,
                                                                 0);
      }
    }
  };
  // ROLL: the rolling prefetch where the full second fragment set spilled, the 128-column
  // 64-channel-chunk residual-forward and gate-out items (12-36 B/lane at 255 VGPRs,
  // round 4; without any prefetch they run 4-7 % longer, profiles/r05_spill_*)
  constexpr bool ROLL = BN == 128 && CK == 64 && (GOK || EP == EP_FWD_RES);
  // (the gate-out residual form, which the train step does not launch, spills even so:
  // no prefetch there)
  constexpr bool NOPF = BN == 128 && CK == 64 && GOK && EP == EP_RES;
  auto compute = [&](int jj, const unsigned char* ph, const unsigned char* pbs) {
    if constexpr (NOPF) compute_np(jj, ph, pbs);
    else if constexpr (ROLL) compute_roll(jj, ph, pbs);
    else compute_pf(jj, ph, pbs);
  };

  // ---- epilogue: straight from the accumulators, through buffer descriptors on the
  // item's first pixel (32-bit offsets: few registers; pixels past the image edge get
  // the OOB offset, so loads read zeros and stores are dropped, no branches).  Lane
  // (r, g) of fragment (i, jn) holds channels cl..cl+3 of tile pixel (row wm*MT + i,
  // column r): one 8-byte unit per operand.
  u32x2 eop[(RES || ACC) ? MT : 1][(RES || ACC) ? NTL : 1];
  u32x2 gpre[GOK ? MT : 1][GOK ? NTL : 1];
  // epilogue operands (residual / accumulate target / gated layer's PReLU input),
  // issued at the epilogue's start (issuing them at the start of the item's last K
  // stage instead made the 80-column level-1 input gradient 67 -> 72 us: that
  // stage's closing vmcnt(0) then waits on an HBM round trip)
  auto epi_load = [&](const Geo& q) {
    const int64_t pix0 = ((int64_t)q.nimg * H + q.y0) * W + q.x0;
    const bool col_ok = q.x0 + r < W;
    if constexpr ((RES || ACC) && W16) {   // one 16-byte unit per (row pair, n-tile): [2p] low, [2p+1] high
      const int ops = (int)d.out_ps;
      const int eps = RES ? (int)d.res_ps : ops;
      const __amdgpu_buffer_rsrc_t re =
          rdn_rsrc(RES ? (const bf16*)d.res + pix0 * d.res_ps : (const bf16*)d.out + pix0 * d.out_ps);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        const int cl = q.n0 + wn * WTN + jn * 16 + 8 * (g >> 1);
        const int coff =
            RES ? rdn_coff32(d.res_c0 + cl, eps, (int)d.res_pl) : rdn_coff32(d.out_c0 + cl, ops, (int)d.out_pl);
        const bool cok = col_ok & (RES ? cl < d.res_climit : true);
#pragma unroll
        for (int p = 0; p < MT / 2; ++p) {
          const int i = 2 * p + (g & 1);
          const bool ok = cok & (q.y0 + wm * MT + i < H);
          const u32x4 u = rdn_ld16(re, ok, (((wm * MT + i) * W + r) * eps + coff) * 2);
          eop[2 * p][jn] = u32x2{u[0], u[1]};
          eop[2 * p + 1][jn] = u32x2{u[2], u[3]};
        }
      }
    } else if constexpr (RES || ACC) {
      const int ops = (int)d.out_ps;
      const int eps = RES ? (int)d.res_ps : ops;
      const __amdgpu_buffer_rsrc_t re =
          rdn_rsrc(RES ? (const bf16*)d.res + pix0 * d.res_ps : (const bf16*)d.out + pix0 * d.out_ps);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        const int cl = q.n0 + wn * WTN + jn * 16 + g * 4;
        const int coff =
            RES ? rdn_coff32(d.res_c0 + cl, eps, (int)d.res_pl) : rdn_coff32(d.out_c0 + cl, ops, (int)d.out_pl);
        const bool cok = col_ok & (RES ? cl < d.res_climit : true);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bool ok = cok & (q.y0 + wm * MT + i < H);
          eop[i][jn] = rdn_ld8(re, ok, (((wm * MT + i) * W + r) * eps + coff) * 2);
        }
      }
    }
    if constexpr (GOK) {   // saved PReLU input of the gated columns
      const __amdgpu_buffer_rsrc_t rg = rdn_rsrc((const bf16*)d.gout_pre + pix0 * d.gout_pre_ps);
      const int gps = (int)d.gout_pre_ps;
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        const int cl = q.n0 + wn * WTN + jn * 16 + g * 4;
        const bool gok = col_ok & (cl >= d.gout_c0);
#pragma unroll
        for (int i = 0; i < MT; ++i)
          gpre[i][jn] = rdn_ld8(rg, gok & (q.y0 + wm * MT + i < H), (((wm * MT + i) * W + r) * gps + cl - d.gout_c0) * 2);
      }
    }
  };
  // W16 epilogue: rows 2p, 2p+1 of a wave's pixel rows exchanged between lane rows
  // g, g^1: lane (r, g) finishes channels cl..cl+7 of pixel row 2p + (g & 1)
  auto epilogue16 = [&](const Geo& q) {
    epi_load(q);
    const int64_t pix0 = ((int64_t)q.nimg * H + q.y0) * W + q.x0;
    const __amdgpu_buffer_rsrc_t ro = rdn_rsrc((const bf16*)d.out + pix0 * d.out_ps);
    const int ops = (int)d.out_ps, pps = (int)d.pre_ps;
    const bool col_ok = q.x0 + r < W;
    const __amdgpu_buffer_rsrc_t rp = FWD && spre ? rdn_rsrc((const bf16*)d.pre + pix0 * d.pre_ps) : ro;
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) {
      const int cl = q.n0 + wn * WTN + jn * 16 + 8 * (g >> 1);
      f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0, a0 = b0, a1 = b0;
      if constexpr (FWD) {
        b0 = *(const f32x4*)(tab + cl);
        b1 = *(const f32x4*)(tab + cl + 4);
        a0 = *(const f32x4*)(tab + COL_MAX + cl);
        a1 = *(const f32x4*)(tab + COL_MAX + cl + 4);
      }
      const int co = rdn_coff32(d.out_c0 + cl, ops, (int)d.out_pl);
      const int cp = FWD ? rdn_coff32(cl, pps, (int)d.pre_pl) : 0;
      const bool res_ok = RES ? cl < d.res_climit : true;
#pragma unroll
      for (int p = 0; p < MT / 2; ++p) {
        const int i = 2 * p + (g & 1);
        const bool ok = col_ok & (q.y0 + wm * MT + i < H);
        const int prow = (wm * MT + i) * W + r;
        // (whole-vector bit casts only: rdn_common.h's note on ext_vector elements)
        const u32x4 ua = __builtin_bit_cast(u32x4, acc[2 * p][jn]), ub = __builtin_bit_cast(u32x4, acc[2 * p + 1][jn]);
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
          v[e] = flo[e];
          v[4 + e] = fhi[e];
        }
        if constexpr (FWD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] += b0[e];
            v[4 + e] += b1[e];
          }
          int o = ok && spre ? (prow * pps + cp) * 2 : RDN_OOB;
          asm volatile("" : "+v"(o));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, Unit16<bf16>::pack(v)), rp, o, 0, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = v[e] > 0.f ? v[e] : a0[e] * v[e];
            v[4 + e] = v[4 + e] > 0.f ? v[4 + e] : a1[e] * v[4 + e];
          }
        }
        if constexpr (RES || ACC) {
          if (res_ok) {
            v[0] += bf16lo(eop[2 * p][jn][0]); v[1] += bf16hi(eop[2 * p][jn][0]);
            v[2] += bf16lo(eop[2 * p][jn][1]); v[3] += bf16hi(eop[2 * p][jn][1]);
            v[4] += bf16lo(eop[2 * p + 1][jn][0]); v[5] += bf16hi(eop[2 * p + 1][jn][0]);
            v[6] += bf16lo(eop[2 * p + 1][jn][1]); v[7] += bf16hi(eop[2 * p + 1][jn][1]);
          }
        }
        int o = ok ? (prow * ops + co) * 2 : RDN_OOB;
        asm volatile("" : "+v"(o));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, Unit16<bf16>::pack(v)), ro, o, 0, 0);
      }
    }
  };
  auto epilogue = [&](const Geo& q, int itm) {
    if constexpr (W16) {
      (void)itm;
      epilogue16(q);
      return;
    }
    epi_load(q);
    const int64_t pix0 = ((int64_t)q.nimg * H + q.y0) * W + q.x0;
    const __amdgpu_buffer_rsrc_t ro = rdn_rsrc((const bf16*)d.out + pix0 * d.out_ps);
    const __amdgpu_buffer_rsrc_t rgo = GOK ? rdn_rsrc((const bf16*)d.gout + pix0 * d.gout_ps) : ro;
    const int ops = (int)d.out_ps, pps = (int)d.pre_ps;
    const bool col_ok = q.x0 + r < W;
    const __amdgpu_buffer_rsrc_t rp = FWD && spre ? rdn_rsrc((const bf16*)d.pre + pix0 * d.pre_ps) : ro;
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) {
      const int cl = q.n0 + wn * WTN + jn * 16 + g * 4;
      f32x4 bias = {0.f, 0.f, 0.f, 0.f}, alpha = {0.f, 0.f, 0.f, 0.f};
      if constexpr (FWD) {
        bias = *(const f32x4*)(tab + cl);
        alpha = *(const f32x4*)(tab + COL_MAX + cl);
      }
      const int co = rdn_coff32(d.out_c0 + cl, ops, (int)d.out_pl);
      const int cp = FWD ? rdn_coff32(cl, pps, (int)d.pre_pl) : 0;
      const bool res_ok = RES ? cl < d.res_climit : true;
      float gsa[4] = {0.f, 0.f, 0.f, 0.f}, gsb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const bool ok = col_ok & (q.y0 + wm * MT + i < H);
        const int prow = (wm * MT + i) * W + r;   // pixel relative to the item origin
        float v[4] = {acc[i][jn][0], acc[i][jn][1], acc[i][jn][2], acc[i][jn][3]};
        if constexpr (FWD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bias[e];
          int o = ok && spre ? (prow * pps + cp) * 2 : RDN_OOB;
          asm volatile("" : "+v"(o));
          __builtin_amdgcn_raw_buffer_store_b64(rdn_pack4(v), rp, o, 0, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : alpha[e] * v[e];
        }
        if constexpr (RES || ACC) {
          if (res_ok) {
            v[0] += bf16lo(eop[i][jn][0]); v[1] += bf16hi(eop[i][jn][0]);
            v[2] += bf16lo(eop[i][jn][1]); v[3] += bf16hi(eop[i][jn][1]);
          }
        }
        if constexpr (GOK) {
          if (cl >= d.gout_c0) {   // complete dY of the gated layer: store its dYpre instead
            const int gc = cl - d.gout_c0;
            const f32x4 al = *(const f32x4*)(tab + COL_MAX + gc);
            const float pr[4] = {bf16lo(gpre[i][jn][0]), bf16hi(gpre[i][jn][0]), bf16lo(gpre[i][jn][1]),
                                 bf16hi(gpre[i][jn][1])};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bool pos = pr[e] > 0.f;
              if (ok && !pos) gsa[e] += pr[e] * v[e];
              v[e] = pos ? v[e] : al[e] * v[e];
              if (ok) gsb[e] += v[e];
            }
            int o = ok ? (prow * (int)d.gout_ps + gc) * 2 : RDN_OOB;
            asm volatile("" : "+v"(o));
            __builtin_amdgcn_raw_buffer_store_b64(rdn_pack4(v), rgo, o, 0, 0);
            continue;
          }
        }
        int o = ok ? (prow * ops + co) * 2 : RDN_OOB;
        asm volatile("" : "+v"(o));
        __builtin_amdgcn_raw_buffer_store_b64(rdn_pack4(v), ro, o, 0, 0);
      }
      if constexpr (GOK) {
        if (cl >= d.gout_c0) {   // this 16-lane group's channel partials over the item's pixels
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int m = 1; m < 16; m <<= 1) {
              gsa[e] += __shfl_xor(gsa[e], m, 64);
              gsb[e] += __shfl_xor(gsb[e], m, 64);
            }
          if (r == 0) {
            const int gcn = d.ncols - d.gout_c0;
            float* const prt = d.gout_part + ((int64_t)(itm / ncb) * WM + wm) * 2 * gcn + (cl - d.gout_c0);
            *(f32x4*)prt = f32x4{gsa[0], gsa[1], gsa[2], gsa[3]};
            *(f32x4*)(prt + gcn) = f32x4{gsb[0], gsb[1], gsb[2], gsb[3]};
          }
        }
      }
    }
  };

  // ---- prologue: first item's chunk-0 halo and first weight stage
  Geo cur = geo(item < it_hi ? item : it_lo);
  if (item < it_hi) {
    issue_w(cur.n0, 0, 0, 0);
    issue_h(cur, 0, 0);
  }
  wait_vm<0>();
  __syncthreads();   // slopes / biases, first halo and weights
  // Per LDS stage: issue the NEXT weight stage (into the buffer every wave finished
  // reading before the last barrier) and, at a chunk's first stage, the next chunk's
  // halo (into the other halo buffer, free since the chunk boundary's barrier), then
  // compute; each wave then waits for its own weight DMA of the next stage -- the
  // halo DMA issued after it stays in flight one more stage -- and a barrier
  // publishes the stage.  Epilogue stores go out right after the item's last barrier
  // and are retired by the next stage's wait.
  int wbuf = 0, hbuf = 0;
  while (item < it_hi) {
    const int nxt_item = item + per;
    const bool has_next = nxt_item < it_hi;
    const Geo nq = geo(has_next ? nxt_item : item);
    zero_acc();
    for (int c = 0; c < nch; ++c) {
      const bool more = c + 1 < nch;
      const unsigned char* const ph = halo + hbuf * Cfg::HALO_BYTES;
#pragma unroll
      for (int jj = 0; jj < SS; ++jj) {
        const bool nxt = jj + 1 < SS || more || has_next;
#ifdef BIG_DIAG_NO_DMA   // diagnostic build (timing only): the prologue's stage and halo only
        if (false) {
#else
        if (nxt) {
#endif
          if (jj + 1 < SS) issue_w(cur.n0, c, jj + 1, wbuf ^ 1);
          else if (more) issue_w(cur.n0, c + 1, 0, wbuf ^ 1);
          else issue_w(nq.n0, 0, 0, wbuf ^ 1);
        }
#ifdef BIG_DIAG_NO_DMA
        const bool hl = false;
#else
        const bool hl = jj == 0 && (more || has_next);
#endif
        if (hl) issue_h(more ? cur : nq, more ? c + 1 : 0, hbuf ^ 1);
        compute(jj, ph, wst + wbuf * Cfg::W_BYTES + b_lane);
#ifndef BIG_DIAG_NO_BAR   // diagnostic build (timing only): no per-stage wait and barrier
        if (hl && SS > 1) wait_split<HP / NW, HP / NW + 1, HP % NW>(wave);   // weights landed; halo may fly
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
#endif
        asm volatile("" ::: "memory");
        wbuf ^= 1;
      }
      hbuf ^= 1;
    }
#ifdef BIG_DIAG_NO_EPI   // diagnostic build (timing only): one conditional store keeps the accumulators live
    {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) t += acc[i][jn][0] + acc[i][jn][3];
      if (t == 1.2345f) ((float*)d.out)[tid] = t;
    }
#else
    epilogue(cur, item);   // global stores drain under the next item
#endif
    item = nxt_item;
    cur = nq;
  }
}

int big_mode() {
  // RDN_BIG: unset/"1" = the default shape rule below; "0" = never (conv3_halo)
  static const int m = [] {
    const char* e = getenv("RDN_BIG");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return m;
}

int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8) n = 256;
    cus = n;
  }
  return cus;
}

int epi_mode(const rdn_conv_desc* d) {
  // (a forward-only engine keeps no PReLU input: its pre stores go to the OOB offset,
  // which the buffer descriptor drops -- round 6, the samplers' level-1..3 convs had
  // fallen back to conv3_halo)
  const int f = d->flags & ~RDN_EPI_STORE_PRE;
  const int fwd = RDN_EPI_BIAS | RDN_EPI_PRELU;
  if (f == fwd) return EP_FWD;
  if (f == (fwd | RDN_EPI_RESID)) return EP_FWD_RES;
  if (d->flags & RDN_EPI_STORE_PRE) return -1;
  if (f == 0) return EP_PLAIN;
  if (f == RDN_EPI_ACCUM) return EP_ACC;
  if (f == RDN_EPI_RESID) return EP_RES;
  return -1;
}

template <int TH, int BN, int WM, int CK, int EP, bool GO = false, int NW = 8>
int launch_pt(const rdn_conv_desc* d, hipStream_t st, int tiles_x, int tiles_y, int nitems) {
  using Cfg = PtCfg<TH, BN, WM, CK, NW>;
  if constexpr (!Cfg::OK) {
    return 1;
  } else {
    constexpr bool FWD_ = EP == EP_FWD || EP == EP_FWD_RES;
    if constexpr (!(GO && !FWD_) && Cfg::MT % 2 == 0) {
      // 16-byte epilogue units: 8-channel aligned operands
      auto a8 = [](int64_t ps, int64_t c0, const void* p) { return ps % 8 == 0 && c0 % 8 == 0 && !((uintptr_t)p & 15); };
      if (!a8(d->out_ps, d->out_c0, d->out)) return 1;
      if (FWD_ && !a8(d->pre_ps, 0, d->pre)) return 1;
      if ((EP == EP_FWD_RES || EP == EP_RES) && (!a8(d->res_ps, d->res_c0, d->res) || d->res_climit % 8)) return 1;
    }
    if (GO) rdn_probe_rows = (int)((int64_t)d->n * tiles_x * tiles_y * WM);
    RDN_PROBE("conv3_big_kernel<bf16,%d,%d,%d,%d%s%s>", TH, BN, WM, CK, GO ? ",go" : "", NW == 4 ? ",w4" : "");
    const int per_xcd = (nitems + 7) / 8;
    int slots = Cfg::BPC * cu_count() / 8;   // blocks per XCD
    if (slots > per_xcd) slots = per_xcd;
    if (slots < 1) slots = 1;
    hipLaunchKernelGGL((conv3_big_kernel<TH, BN, WM, CK, EP, GO, NW>), dim3((unsigned)(8 * slots)), dim3(Cfg::NTB), 0,
                       st, *d, tiles_x, tiles_y, nitems);
    return rdn_check_launch("rdn_conv_fwd(conv3 big)");
  }
}

template <int TH, int BN, int WM, int CK, int NW = 8>
int launch_big(const rdn_conv_desc* d, hipStream_t st) {
  const int tiles_x = (d->w + TWB - 1) / TWB, tiles_y = (d->h + TH - 1) / TH;
  const int64_t nitems = (int64_t)d->n * tiles_x * tiles_y * (d->ncols / BN);
  if (nitems >= (1ll << 31)) return 1;
  const int ni = (int)nitems;
  if (d->gout) {   // gate-out: the input-gradient modes only (8-wave blocks: the 4-wave ones spill)
    if constexpr (NW == 8) {
      switch (epi_mode(d)) {
        case EP_PLAIN: return launch_pt<TH, BN, WM, CK, EP_PLAIN, true>(d, st, tiles_x, tiles_y, ni);
        case EP_ACC: return launch_pt<TH, BN, WM, CK, EP_ACC, true>(d, st, tiles_x, tiles_y, ni);
        case EP_RES: return launch_pt<TH, BN, WM, CK, EP_RES, true>(d, st, tiles_x, tiles_y, ni);
      }
    }
    return 1;
  }
  switch (epi_mode(d)) {
    case EP_FWD: return launch_pt<TH, BN, WM, CK, EP_FWD, false, NW>(d, st, tiles_x, tiles_y, ni);
    case EP_FWD_RES: return launch_pt<TH, BN, WM, CK, EP_FWD_RES, false, NW>(d, st, tiles_x, tiles_y, ni);
    case EP_PLAIN: return launch_pt<TH, BN, WM, CK, EP_PLAIN, false, NW>(d, st, tiles_x, tiles_y, ni);
    case EP_ACC: return launch_pt<TH, BN, WM, CK, EP_ACC, false, NW>(d, st, tiles_x, tiles_y, ni);
    case EP_RES: return launch_pt<TH, BN, WM, CK, EP_RES, false, NW>(d, st, tiles_x, tiles_y, ni);
  }
  return 1;
}

// Where the persistent kernel wins (per-layer A/B against conv3_halo on the train
// step's own launches, B16 and B32, profiles/r03_v3_big_vs_halo.json):
// * items spread evenly over the CUs (the last round >= 90 % full: one item more on
//   some CUs is a whole item of tail, where conv3_halo's 128-pixel tiles at 2-3
//   blocks per CU balance finer);
// * 128 / 96-column items (64 x 64 / 64 x 48 wave tiles) with >= 2 channel chunks
//   per item, or >= 4 items per CU on >= 128 x 128 images (with one chunk and one
//   item per CU the next halo's load is exposed); 80 / 64-column items (32 x 80 /
//   64 x 32 wave tiles, LDS-read heavier) with >= 8 chunk iterations per CU on
//   >= 128 x 128 images, where the cross-item prefetch carries them (the level-1
//   input gradients: 20-35 % faster than conv3_halo, up_0's 1.6x);
// * 32-channel chunks: single-chunk input gradients and (round 4, with the k-step
//   prefetch) the 5-chunk 160-channel level-1 conv_3 forward (big_ck32_multi).
// multi-chunk 32-channel items: the 160-channel level-1 conv_3 forward (5 chunks; it
// lost to conv3_halo in round 3, before the k-step prefetch; round 4, interleaved:
// 82 -> 74 us per launch, step +0.5 % B16 / +0.4 % B32, profiles/r04_v13_big_ck32_ab.txt).
// RDN_BIG_CK32=0: single-chunk 32-channel items only (A/B)
bool big_ck32_multi() {
  static const bool on = [] {
    const char* e = getenv("RDN_BIG_CK32");
    return !(e && e[0] == '0');
  }();
  return on;
}

// RDN_BIG_NW4=0: the 64-column 32-channel-chunk items on 8-wave blocks (A/B)
bool big_nw4() {
  static const bool on = [] {
    const char* e = getenv("RDN_BIG_NW4");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool big_fall() {
  static const bool on = [] {
    const char* e = getenv("RDN_BIG_FALL");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int CK>
int big_dispatch(const rdn_conv_desc* d, hipStream_t st) {
  const int64_t tiles = (int64_t)d->n * ((d->h + 15) / 16) * ((d->w + 15) / 16);
  const int cus = cu_count(), nch = d->cin / CK;
  if (CK == 32 && nch != 1 && !big_ck32_multi()) return 1;
  auto even = [&](int64_t items) {
    const int64_t rounds = (items + cus - 1) / cus;
    return items >= cus && items * 10 >= rounds * cus * 9;
  };
  // single-chunk and narrow-column launches won on the >= 128 x 128 images (level 1,
  // up_0) and lost on level 2's 64 x 64 ones (r03 per-layer A/B)
  const bool big_img = (int64_t)d->h * d->w >= 128 * 128;
  // Round 4 (with the k-step prefetch), per-layer A/B on the train step at B16 / B32
  // (profiles/r04_v14_big_loose_layers.txt): the 128-column items now win on any evenly
  // spread grid (level-2 conv_2 input gradient 55 -> 48 / 104 -> 88 us, conv_0 -3 / -5
  // us) and so do the 64-column ones (level-2 conv_0..2 forward -1..-2 / -6..-13 us);
  // the 96-column (conv_1 dgrad: even) and 80-column ones (conv_3 dgrad: +4 / +16 us)
  // keep the round-3 rule.  RDN_BIG_LOOSE=0: the round-3 rule everywhere.
  static const bool loose = [] {
    const char* e = getenv("RDN_BIG_LOOSE");
    return !(e && e[0] == '0');
  }();
  auto wide_ok = [&](int bn) {
    const int64_t items = tiles * (d->ncols / bn);
    return even(items) && ((loose && bn == 128) || nch >= 2 || (items >= 4ll * cus && big_img));
  };
  auto narrow_ok = [&](int bn) {
    const int64_t items = tiles * (d->ncols / bn);
    return even(items) && ((loose && bn == 64) || (items * nch >= 8ll * cus && big_img));
  };
  if (d->ncols % 128 == 0) return wide_ok(128) ? launch_big<16, 128, 4, CK>(d, st) : 1;
  if (d->ncols % 96 == 0) return wide_ok(96) ? launch_big<16, 96, 4, CK>(d, st) : 1;
  if (d->ncols % 80 == 0) {
    if (narrow_ok(80)) return launch_big<16, 80, 8, CK>(d, st);
    // the 320-column level-2 conv_3 input gradient on 64-column items (<= 6 per CU):
    // faster alone (B16 72-77 -> 67-69 us, profiles/r04_v17_big_fall_layers.txt) but
    // slower in the step beside the weight-gradient stream (1715 -> 1708 img/s,
    // interleaved, r04_v18_big_fall_ab.txt); after round 6's changes faster at B16 in
    // five of five interleaved rounds (1858 -> 1871 img/s, B32 2062 -> 2047,
    // profiles/r06_big_fall_ab.txt): on, RDN_BIG_FALL=0 for the conv3_halo fallback
    if (!(big_fall() && d->ncols % 64 == 0 && tiles * (d->ncols / 64) <= 6ll * cus)) return 1;
  }
  if (d->ncols % 64 == 0) {
    if (!narrow_ok(64)) return 1;
    if constexpr (CK == 32)   // two 4-wave blocks per CU (79 KB of LDS each), 64 x 64 wave tiles
      if (big_nw4() && !d->gout) return launch_big<16, 64, 4, CK, 4>(d, st);
    return launch_big<16, 64, 4, CK>(d, st);
  }
  if (d->ncols == 32) {
    // the narrow level-1 forwards (64 / 128 input channels -> 32; 32 x 32 wave tiles,
    // near the HBM ridge): per-layer A/B at B16, conv_0 28 -> 26 us (was conv3_wsd),
    // conv_2 41 -> 36.5 us (was conv3_halo); the 32-channel level-0 ones are a tie
    // with conv3_ws and stay there
    if constexpr (CK == 64) {
      const int64_t items = tiles;
      return (even(items) && items >= 4ll * cus && big_img) ? launch_big<16, 32, 8, CK>(d, st) : 1;
    }
  }
  return 1;
}

}  // namespace

// Level 1-3 bf16 3x3 convs with enough columns and input channels for the large
// tile (else 1: the caller falls back to conv3_wsd / conv3_ws / conv3_halo)
int rdn_conv3_big_launch(const rdn_conv_desc* d, int ck, hipStream_t st) {
  if (!big_mode() || d->dtype != RDN_BF16 || d->gather != RDN_G_CONV3) return 1;
  if (d->bn || d->bm || d->gate) return 1;
  if (ck != 32 && ck != 64) return 1;
  if (epi_mode(d) < 0) return 1;
  if (d->ncols % 16 || d->ncols < 32 || d->cin < 32 || d->ncols > COL_MAX) return 1;
  if (d->x_ps % 8 || d->x_c0 % 8 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15) || d->kp % 8) return 1;
  if (d->out_ps % 4 || d->out_c0 % 4 || ((uintptr_t)d->out & 7)) return 1;
  if ((d->flags & RDN_EPI_STORE_PRE) && (d->pre_ps % 4 || ((uintptr_t)d->pre & 7))) return 1;
  if ((d->flags & RDN_EPI_RESID) && (d->res_ps % 4 || d->res_c0 % 4 || d->res_climit % 4 || ((uintptr_t)d->res & 7)))
    return 1;
  // grids of at least one item per CU at the 16 x 16 x 128 tile (levels 1-3 of the
  // 256^2 train step and larger)
  const int64_t px = (int64_t)d->n * d->h * d->w;
  if (px < 8192) return 1;
  // 32-bit element offsets (halo) and byte offsets (epilogue, from a per-item base)
  auto fits = [&](int64_t ps, int64_t pl, int c_hi) {
    return 2 * ((int64_t)(18 + 1) * d->w * ps + rdn_coff(c_hi, ps, pl)) < (int64_t)RDN_OOB - 16;
  };
  if (!fits(d->x_ps, d->x_pl, d->x_c0 + d->cin) || !fits(d->out_ps, d->out_pl, d->out_c0 + d->ncols) ||
      ((d->flags & RDN_EPI_STORE_PRE) && !fits(d->pre_ps, d->pre_pl, d->ncols)) ||
      ((d->flags & RDN_EPI_RESID) && !fits(d->res_ps, d->res_pl, d->res_c0 + d->res_climit)))
    return 1;
  if (d->gout && (d->ncols - d->gout_c0 > COL_MAX || d->gout_c0 % 4 || d->gout_ps % 4 || d->gout_pre_ps % 4 ||
                  !fits(d->gout_ps, 0, d->ncols - d->gout_c0) || !fits(d->gout_pre_ps, 0, d->ncols - d->gout_c0) ||
                  ((uintptr_t)d->gout_part & 15)))
    return 1;
  return ck == 64 ? big_dispatch<64>(d, st) : big_dispatch<32>(d, st);
}
