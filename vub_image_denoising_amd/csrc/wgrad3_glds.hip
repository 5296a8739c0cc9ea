// Weight gradient of the 3x3 / pad 1 convolutions, LDS-DMA pipelined (gfx950):
//
//   ws[split][co][tap*ndim + ci] = sum_p dYpre[p][co] * X[p + tap][ci]
//
// Same decomposition as wgrad3_rows_kernel (wgrad3_halo.hip): a block owns BM
// output channels x one CK-channel group x a range of 8 x 16 pixel tiles (split-K
// over pixels), the dYpre tile [128 px][BM] and the input halo [10 x 18 px][CK]
// of a tile feed all 9 taps from LDS.  What differs is the staging: the rows
// kernel moves each tile global -> VGPR -> LDS with ONE tile in flight, so at the
// level-2/3 shapes (one or two blocks per CU) it waits on load latency most of the
// time (r02: 0.15-0.18 of the bf16 MFMA peak, ~4 B/clk/CU of L2 traffic).  Here
// every tile goes straight to LDS with global_load_lds_dwordx4 (no VGPR staging)
// into a ring of NS = 3 LDS stages: while tile t is multiplied, tiles t+1 and t+2
// are in flight.  Each wave waits only for its own DMAs with a counted
// `s_waitcnt vmcnt` and a raw s_barrier publishes them (an LDS-DMA is a pending
// write on the VM counter, so __syncthreads() would drain the whole ring:
// cdna_hip_programming.md §5 "Pipelining across barriers").  The barrier also
// retires the reads of the stage the next DMA overwrites (it was read one tile
// earlier).
//
// Multi-chunk (level-1..3) launches only: the single-chunk level-0/1 weight
// gradients, where the PReLU backward is fused into the loader, stay on the rows
// kernel (a gated variant of this one was faster alone but its one 135-KB block per
// CU on the weight-gradient stream cost the dgrad chain more: 1490 vs 1497 img/s, r02).
//
// LDS images.  One DMA wave-instruction writes 1 KiB contiguously (lane l ->
// bytes l*16..l*16+15), so the images are dense rows (dY: BM*2 bytes per pixel;
// halo: CK*2 bytes per pixel) and bank conflicts of the ds_read_b64_tr_b16
// fragment reads are removed by rotating each row's 16-byte units by rot(x),
// x = the pixel's column in its tile row (0..15) or halo row (0..17), applied on
// the per-lane SOURCE address (rotations from an exhaustive check of the read
// patterns: conflict-free for every row size used).  Because the rotation depends
// on the column only, every fragment address is a per-lane base fixed for the
// launch plus an immediate.
//
// Pixels outside the image (partial tiles, halo borders) and channels past mdim
// load 16 zero bytes from a device-side zero block, so stale stage bytes never
// reach the MFMAs.
#include "rdn_common.h"


#include <type_traits>

namespace {

__device__ __attribute__((aligned(64))) unsigned int g_wglds_zero[16];

constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HW_ = TW + 2, HP = (TH + 2) * HW_;
constexpr int LDS_MAX = 160 * 1024;


template <int BM, int CK>
struct Geo {
  // waves per block: 8 (two per SIMD) -- while one wave issues its LDS-DMA pieces or
  // waits on LDS the other multiplies.  r03: 64 x 64 shapes only (64 x 72 wave tiles,
  // 218 VGPRs, 6-8 % faster per launch, profiles/r03_v10_wgrad_glds_diag.txt); the 80-
  // and 96-column groups spilled there, because every k-step's B fragments (NTW of
  // them, double-buffered) were read ahead at once.  Round 4: a (k-step, n-tile)
  // software pipeline with only a few B fragments live, so every shape fits two waves
  // per SIMD -- bit-identical, but 1-6 % slower per launch on 5 of the 7 train-step
  // shapes and -0.5 % on the step (profiles/r04_v4_wgrad_pipe_*).  Round 5: 4-wave
  // blocks with 64 x 144 AGPR wave tiles for 64 x 64 ran 93 -> 100 us
  // (profiles/r05_wgrad_agpr_kbench_ab.txt).  Neither kept.
  static constexpr int NW = (BM == 64 && CK == 64) ? 8 : 4,
                       NTH = 64 * NW;   // (64 x 96: 78 VGPRs of spill at two waves per SIMD)
  static constexpr int NCOL = 9 * CK, NT_ALL = (NCOL + 15) / 16;
  // waves as WMv (along M) x WNv (along the 9*CK columns), the same number of
  // n-tiles for every wave (a wave-dependent trip count costs accumulator copies);
  // n-tiles past NT_ALL are computed on a valid column and not stored
  static constexpr int WNv = (BM == 64 && NT_ALL % 4 != 0) ? 2 : 4, WMv = NW / WNv;
  static constexpr int NTW = (NT_ALL + WNv - 1) / WNv;    // n-tiles per wave
  static constexpr int MTW = BM / 16 / WMv;               // 16-row m-tiles per wave
  static constexpr int RA = BM * 2, RB = CK * 2;          // bytes per dY / halo pixel row
  static constexpr int UA = RA / 16, UB = RB / 16;        // 16-B units per row
  static constexpr int A_PIECES = TP * RA / 1024;
  static constexpr int PA = A_PIECES / NW;                // dY pieces per wave and tile
  static constexpr int HPC = (HP * RB + 1023) / 1024;     // halo pieces (wave w: w, w+4, ...)
  static constexpr int HPW = (HPC + NW - 1) / NW;
  static constexpr int B_OFF = A_PIECES * 1024;
  static constexpr int STAGE = B_OFF + HPC * 1024;
  static constexpr int NS = 3 * STAGE <= LDS_MAX ? 3 : 2;   // (4 stages where they fit: no change, r03)
  static constexpr bool OK = NS * STAGE <= LDS_MAX && MTW >= 1;
  static_assert(A_PIECES % NW == 0 && CK % 8 == 0, "image geometry");
};

// unit rotation of a RBYTES-byte image row at column x (bank-conflict-free
// ds_read_b64_tr_b16 of 8 consecutive columns x one 32-byte unit pair)
template <int RBYTES>
__device__ __forceinline__ int rot(int x) {
  constexpr int U = RBYTES / 16;
  if constexpr (RBYTES == 64) return (x >> 1) % U;
  else if constexpr (RBYTES == 128) return x % U;
  else if constexpr (RBYTES == 192) return ((x >> 2) * 6) % U;
  else if constexpr (RBYTES == 256) return x % U;
  else return 0;                                          // 32, 96, 160: conflict-free as is
}

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// DMAs wave w issues per tile: PA_ dY pieces + halo pieces w, w+4, ... < HPC;
// wait until at most `ahead` later tiles of this wave's DMAs are in flight
template <int PA_, int HPC, int NW, int K, int W = 0>
__device__ __forceinline__ void wait_own_k(int wave) {   // wave w issues PA_ + (HPC - w + NW - 1) / NW per tile
  if constexpr (W < NW - 1) {
    if (wave == W) { wait_vm<K * (PA_ + (HPC + NW - 1 - W) / NW)>(); return; }
    wait_own_k<PA_, HPC, NW, K, W + 1>(wave);
  } else {
    wait_vm<K * (PA_ + (HPC + NW - 1 - W) / NW)>();
  }
}
template <int PA_, int HPC, int NW>
__device__ __forceinline__ void wait_own(int wave, int ahead) {
  if (ahead <= 0) wait_vm<0>();
  else if (ahead == 1) wait_own_k<PA_, HPC, NW, 1>(wave);
  else wait_own_k<PA_, HPC, NW, 2>(wave);
}

// One LDS-DMA wave-instruction: 16 B per lane from `src` to LDS byte dst + lane*16
// (dst wave-uniform, in M0).  Inline asm, so that the compiler does not see an
// LDS write pending on the VM counter: with the builtin it waits vmcnt(0) before
// every ds_read of the array, which drains the ring (the counted waits above are
// the only ordering, cdna_hip_programming.md §5, "Read a staged buffer one phase
// AFTER the wait that retires it").
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

template <int BM, int CK>
__global__ __launch_bounds__((Geo<BM, CK>::NTH), 1) void wgrad3_glds_kernel(rdn_wgrad_desc d, int tiles_x, int tiles_y, int ntiles,
                                                             int tiles_per_block) {
  using G_ = Geo<BM, CK>;
  constexpr int RA = G_::RA, RB = G_::RB, UA = G_::UA, UB = G_::UB, NW = G_::NW, MTW = G_::MTW, NTW = G_::NTW;
  constexpr int NS = G_::NS, PA = G_::PA, HPC = G_::HPC, HPW = G_::HPW;
  constexpr int VEC = 8;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NS * G_::STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / G_::WNv, wn = wave % G_::WNv;
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const int mtiles = (d.mdim + BM - 1) / BM, nchunks = d.ndim / CK;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);   // m-tiles, then chunks, of one pixel range share an XCD
  const int bx = lb % mtiles, by = (lb / mtiles) % nchunks, bz = lb / (mtiles * nchunks);
  const int m0 = bx * BM, c0 = by * CK;
  const int t_beg = bz * tiles_per_block;
  const int t_cnt = max(0, min(t_beg + tiles_per_block, ntiles) - t_beg);
  const int H = d.h, W = d.w;
  const bf16* __restrict__ A = (const bf16*)d.a;
  const bf16* __restrict__ Bx = (const bf16*)d.b;
  const bf16* const zero = (const bf16*)g_wglds_zero;

  // ---- per-lane DMA source geometry (tile-invariant)
  int a_rel[PA], a_py[PA], a_px[PA];
  bool a_ok[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int off = (wave + NW * j) * 1024 + lane * 16;
    const int r = off / RA, px = r % TW;
    const int u = ((off % RA) / 16 - rot<RA>(px) + UA) % UA;   // logical unit of this physical slot
    const int m = m0 + u * VEC;
    a_ok[j] = m < d.mdim;
    a_py[j] = r / TW;
    a_px[j] = px;
    a_rel[j] = (a_py[j] * W + px) * (int)d.a_ps + rdn_coff32(d.a_c0 + (a_ok[j] ? m : 0), (int)d.a_ps, (int)d.a_pl);
  }
  int b_rel[HPW], b_hy[HPW], b_hx[HPW];
  bool b_ok[HPW];
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int off = (wave + NW * j) * 1024 + lane * 16;
    const int hr = off / RB, hx = hr % HW_;
    const int u = ((off % RB) / 16 - rot<RB>(hx) + UB) % UB;
    b_ok[j] = hr < HP;
    b_hy[j] = hr / HW_;
    b_hx[j] = hx;
    b_rel[j] = (b_hy[j] * W + hx) * (int)d.b_ps + rdn_coff32(d.b_c0 + c0 + u * VEC, (int)d.b_ps, (int)d.b_pl);
  }

  auto issue = [&](int t, int stage) {
    const int tx = t % tiles_x, r1 = t / tiles_x;
    const int ty = r1 % tiles_y, nimg = r1 / tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;
    const int64_t pix0 = ((int64_t)nimg * H + y0) * W + x0;
    const bool full = y0 + TH <= H && x0 + TW <= W;
    const bool interior = y0 >= 1 && y0 + TH + 1 <= H && x0 >= 1 && x0 + TW + 1 <= W;
    const bf16* const ab = A + pix0 * d.a_ps;
    const bf16* const hb = Bx + (pix0 - W - 1) * d.b_ps;   // halo pixel (0, 0) = image (y0 - 1, x0 - 1)
    const unsigned st = lds_addr(lds) + stage * G_::STAGE;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool ok = a_ok[j] & (full | ((y0 + a_py[j] < H) & (x0 + a_px[j] < W)));
      glds16(ok ? (const void*)(ab + a_rel[j]) : (const void*)zero, st + (wave + NW * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      if (wave + NW * j >= HPC) break;   // wave-uniform
      const bool ok = b_ok[j] & (interior | (((unsigned)(y0 - 1 + b_hy[j]) < (unsigned)H) &
                                             ((unsigned)(x0 - 1 + b_hx[j]) < (unsigned)W)));
      glds16(ok ? (const void*)(hb + b_rel[j]) : (const void*)zero, st + G_::B_OFF + (wave + NW * j) * 1024);
    }
  };

  // ---- per-lane fragment addresses (stage-relative; + immediates per k-step)
  const int xa = 4 * g + q;                               // pixel column of this lane's k rows
  int aoff[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
    aoff[i] = xa * RA + (((wm * (BM / G_::WMv) / 8 + 2 * i + (pp >> 1)) + rot<RA>(xa)) % UA) * 16 + (pp & 1) * 8;
  int boff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wn + G_::WNv * j;
    int c = nt * 16 + 4 * pp;
    c = c < G_::NCOL ? c : 0;                             // padded columns: a valid read, never stored
    const int tp = c / CK, ci = c - tp * CK;
    const int ky = tp / 3, kx = tp - 3 * ky;
    const int hx = xa + kx;
    boff[j] = G_::B_OFF + (ky * HW_ + hx) * RB + (((ci >> 3) + rot<RB>(hx)) % UB) * 16 + (ci & 7) * 2;
  }

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const unsigned char* const st = lds + stage * G_::STAGE;
    // all fragments of k-step ks+1 are read before the MFMAs of ks (at one wave per
    // SIMD nothing else hides the LDS latency; spreading the reads between the MFMAs
    // with sched_group_barrier gained 2-3 %, r03).  Where this wave's time goes (the
    // -DWG_DIAG_* builds, L2 conv_3 at B16): MFMAs alone 38.6 us, + LDS reads 51.2,
    // + LDS-DMA 56.7, everything 66.9 -- the DMA issue and the fragment reads, not the
    // MFMAs, are what the second wave per SIMD (NW = 8) partly hides
    bf16x8 af[2][MTW], bfr[2][NTW];
    auto ld = [&](int ks, int buf) {
#ifdef WG_DIAG_NO_LDS   // diagnostic build (scripts/wg_kbench.py): opaque operands, no LDS reads
#pragma unroll
      for (int i = 0; i < MTW; ++i) asm volatile("" : "=v"(af[buf][i]));
#pragma unroll
      for (int j = 0; j < NTW; ++j) asm volatile("" : "=v"(bfr[buf][j]));
      return;
#endif
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const unsigned char* a = st + aoff[i] + ks * 32 * RA;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, a));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, a + 16 * RA));
        af[buf][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const unsigned char* b = st + boff[j] + ks * 2 * HW_ * RB;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b + HW_ * RB));
        bfr[buf][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    ld(0, 0);
#pragma unroll
    for (int ks = 0; ks < TP / 32; ++ks) {
      if (ks + 1 < TP / 32) ld(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#ifdef WG_DIAG_NO_MFMA   // diagnostic build: fragments consumed without MFMAs
#pragma unroll
      for (int j = 0; j < NTW; ++j) asm volatile("" ::"v"(bfr[ks & 1][j]));
#pragma unroll
      for (int i = 0; i < MTW; ++i) asm volatile("" ::"v"(af[ks & 1][i]));
#else
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int i = 0; i < MTW; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][i], bfr[ks & 1][j], acc[i][j], 0, 0, 0);
#endif
    }
  };

  // ---- NS-deep ring: up to NS-1 tiles in flight while tile it is multiplied;
  // unrolled by NS so that every stage offset is a constant
  for (int k = 0; k < NS - 1; ++k)
    if (k < t_cnt) issue(t_beg + k, k);
  auto step = [&](int it, auto S) {
    constexpr int s = decltype(S)::value;
    // own DMAs of tile it landed (tiles it+1 .. it+NS-2 may still fly)
    wait_own<PA, HPC, NW>(wave, min(NS - 2, t_cnt - 1 - it));
    __builtin_amdgcn_s_barrier();           // everyone's landed; everyone done reading tile it-1's stage
    asm volatile("" ::: "memory");
#ifndef WG_DIAG_NO_DMA   // diagnostic build: only the prologue's tiles are loaded
    if (it + NS - 1 < t_cnt) issue(t_beg + it + NS - 1, (s + NS - 1) % NS);
#endif
    compute(s);
  };
  for (int it = 0; it < t_cnt; it += NS) {
    step(it, std::integral_constant<int, 0>{});
    if (it + 1 < t_cnt) step(it + 1, std::integral_constant<int, 1 % NS>{});
    if constexpr (NS >= 3)
      if (it + 2 < t_cnt) step(it + 2, std::integral_constant<int, 2 % NS>{});
    if constexpr (NS >= 4)
      if (it + 3 < t_cnt) step(it + 3, std::integral_constant<int, 3 % NS>{});
  }

  // D[m][n]: row = g*4 + e (output channel), col = li (tile column)
  const int ncol_all = 9 * d.ndim;
#ifdef WG_DIAG_NO_EPI   // diagnostic build: one store per lane keeps the accumulators live
  {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int i = 0; i < MTW; ++i) t += acc[i][j][0] + acc[i][j][3];
    if (t == 1.2345f) d.ws[threadIdx.x] = t;
    return;
  }
#endif
  float* __restrict__ ws = d.ws + (int64_t)bz * d.mdim * ncol_all;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wn + G_::WNv * j;
    const int c = nt * 16 + li;
    if (nt >= G_::NT_ALL || c >= G_::NCOL) continue;
    const int tp = c / CK, ci = c - tp * CK;
    const int col = tp * d.ndim + c0 + ci;
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * (BM / G_::WMv) + i * 16 + g * 4 + e;
        if (m < d.mdim) ws[(int64_t)m * ncol_all + col] = acc[i][j][e];
      }
  }
}

template <int BM, int CK>
int launch(const rdn_wgrad_desc* d, int blocks, int tiles_x, int tiles_y, int ntiles, int tpb, hipStream_t st) {
  if constexpr (Geo<BM, CK>::OK) {
    if (!d->a_gate) {
      RDN_PROBE("wgrad3_glds_kernel<bf16,%d,%d>", BM, CK);
      wgrad3_glds_kernel<BM, CK><<<blocks, Geo<BM, CK>::NTH, 0, st>>>(*d, tiles_x, tiles_y, ntiles, tpb);
      return rdn_check_launch("rdn_conv_wgrad(conv3 glds)");
    }
  }
  rdn_set_error("rdn_conv_wgrad(conv3 glds): BM=%d CK=%d does not fit", BM, CK);
  return RDN_E_SHAPE;
}

template <int BM>
int launch_ck(const rdn_wgrad_desc* d, int ck, int blocks, int tiles_x, int tiles_y, int ntiles, int tpb,
              hipStream_t st) {
  switch (ck) {
    case 16: return launch<BM, 16>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
    case 32: return launch<BM, 32>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
    case 48: return launch<BM, 48>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
    case 64: return launch<BM, 64>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
    case 80: return launch<BM, 80>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
    case 96: return launch<BM, 96>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
  }
  rdn_set_error("rdn_conv_wgrad(conv3 glds): CK=%d", ck);
  return RDN_E_SHAPE;
}

}  // namespace

// Tile shape of the LDS-DMA weight-gradient kernel for d, or 0 when it does not
// apply.  single_chunk: the rows plan reads the whole input pixel row in one
// channel group (the level-0/1 layers, where the PReLU gate is fused); else the
// multi-chunk (level-1..3) launches.
int rdn_wgrad3_glds_pick(const rdn_wgrad_desc* d, int single_chunk, int* bm, int* ck) {
  if (single_chunk || d->dtype != RDN_BF16 || d->a_gate) return 0;
  if (d->mdim < 32 || d->ndim % 32) return 0;
  *bm = d->mdim <= 32 ? 32 : 64;
  *ck = d->ndim % 64 == 0 ? 64 : 32;
  // the narrow level-1 layers (96 / 128 / 160 input channels): whole-row or half-row
  // channel groups, so operand A (dYpre) is read 1-2 times instead of 2-5 (per-layer
  // A/B, r03_v6: level-1 conv_1 / conv_3 weight gradients -10..-20 %, up_0 -28 %)
  if (d->ndim <= 160) {
    if (d->ndim % 96 == 0) *ck = 96;
    else if (d->ndim % 80 == 0) *ck = 80;   // (128 as one group: 43 -> 45 us, kept at 2 x 64)
  }
  return 1;
}

int rdn_wgrad3_glds_launch(const rdn_wgrad_desc* d, int bm, int ck, int blocks, int tiles_x, int tiles_y, int ntiles,
                           int tpb, hipStream_t st) {
  if (bm == 16) return launch_ck<16>(d, ck, blocks, tiles_x, tiles_y, ntiles, tpb, st);
  if (bm == 32) return launch_ck<32>(d, ck, blocks, tiles_x, tiles_y, ntiles, tpb, st);
  if (bm == 64) return launch_ck<64>(d, ck, blocks, tiles_x, tiles_y, ntiles, tpb, st);
  rdn_set_error("rdn_conv_wgrad(conv3 glds): BM=%d", bm);
  return RDN_E_SHAPE;
}
