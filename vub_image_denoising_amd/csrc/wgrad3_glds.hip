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
// `s_waitcnt vmcnt(G)` and a raw s_barrier publishes them (an LDS-DMA is a
// pending write on the VM counter, so __syncthreads() would drain the whole ring:
// cdna_hip_programming.md §5 "Pipelining across barriers").  The barrier also
// retires the reads of the stage the next DMA overwrites (it was read one tile
// earlier).
//
// LDS images.  One DMA wave-instruction writes 1 KiB contiguously (lane l ->
// bytes l*16..l*16+15), so the images are dense rows (dY: BM*2 bytes per pixel;
// halo: CK*2 bytes per pixel) and bank conflicts of the ds_read_b64_tr_b16
// fragment reads are removed by an XOR swizzle of the 16-byte units applied on the
// per-lane SOURCE address:  unit' = unit ^ 2*s(x),  s(x) = (x / (256/RB)) mod
// (RB/32), where x is the pixel's column inside its tile row (0..15) or halo row
// (0..17).  A half-wave's transpose read touches 8 consecutive columns of one row
// x one 32-byte unit pair; rows that share banks (x and x + 256/RB, ...) get
// distinct unit pairs.  Because s depends on the column only, every fragment
// address is a per-lane base fixed for the launch plus an immediate.
//
// Pixels outside the image (partial tiles, halo borders) load 16 zero bytes from
// a device-side zero block, so stale stage bytes never reach the MFMAs.
#include "rdn_common.h"

#include <cstdlib>
#include <type_traits>

namespace {

__device__ __attribute__((aligned(64))) unsigned int g_wglds_zero[16];

constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HW_ = TW + 2, HP = (TH + 2) * HW_;

template <int BM, int CK>
struct Geo {
  static constexpr int NW = 4, NTH = 256;                // waves per block (one per SIMD)
  static constexpr int NCOL = 9 * CK, NT_ALL = NCOL / 16;
  // waves as WMv (along M) x WNv (along the 9*CK columns) with the same number of
  // n-tiles for every wave (a wave-dependent trip count costs accumulator copies)
  static constexpr int WNv = NT_ALL % 4 == 0 ? 4 : 2, WMv = NW / WNv;
  static constexpr int NTW = NT_ALL / WNv;                // n-tiles per wave
  static constexpr int MTW = BM / 16 / WMv;               // 16-row m-tiles per wave
  static constexpr int RA = BM * 2, RB = CK * 2;         // bytes per dY / halo pixel row
  static constexpr int A_PIECES = TP * RA / 1024;
  static constexpr int PA = A_PIECES / NW;               // dY pieces per wave and tile
  static constexpr int PB = ((HP * RB + 1023) / 1024 + NW - 1) / NW;
  static constexpr int B_PIECES = PB * NW;               // last ones partly padding (zero source)
  static constexpr int STAGE = (A_PIECES + B_PIECES) * 1024;
  static constexpr int G = PA + PB;                      // DMAs per wave and tile (vmcnt unit)
  static_assert(NT_ALL % WNv == 0 && MTW >= 1 && BM % (16 * WMv) == 0, "wave grid");
  static_assert(A_PIECES % NW == 0, "dY pieces split evenly over the waves");
  static_assert(CK % 16 == 0 && RB <= 256 && RA <= 256 && RA >= 64 && RB >= 64, "image geometry");
};

template <int RB>
__device__ __forceinline__ int swz(int x) { return ((x / (256 / RB)) % (RB / 32)) * 2; }

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// One LDS-DMA wave-instruction: 16 B per lane from `src` to LDS byte dst + lane*16
// (dst wave-uniform, in M0).  Inline asm, so that the compiler does not see an
// LDS write pending on the VM counter: with the builtin it waits vmcnt(0) before
// every ds_read of the array, which drains the ring (the counted waits below are
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

template <int BM, int CK, int NS>
__global__ __launch_bounds__(256, 1) void wgrad3_glds_kernel(rdn_wgrad_desc d, int tiles_x, int tiles_y,
                                                                          int ntiles, int tiles_per_block) {
  using G_ = Geo<BM, CK>;
  constexpr int RA = G_::RA, RB = G_::RB, NW = G_::NW, MTW = G_::MTW, NTW = G_::NTW;
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
  int a_rel[G_::PA], a_py[G_::PA], a_px[G_::PA];
  bool a_ok[G_::PA];
#pragma unroll
  for (int j = 0; j < G_::PA; ++j) {
    const int off = (wave + NW * j) * 1024 + lane * 16;
    const int r = off / RA, px = r % TW;
    const int u = ((off % RA) >> 4) ^ swz<RA>(px);
    const int m = m0 + u * 8;
    a_ok[j] = m < d.mdim;
    a_py[j] = r / TW;
    a_px[j] = px;
    a_rel[j] = (a_py[j] * W + px) * (int)d.a_ps + rdn_coff32(d.a_c0 + (a_ok[j] ? m : 0), (int)d.a_ps, (int)d.a_pl);
  }
  int b_rel[G_::PB], b_hy[G_::PB], b_hx[G_::PB];
  bool b_ok[G_::PB];
#pragma unroll
  for (int j = 0; j < G_::PB; ++j) {
    const int off = (wave + NW * j) * 1024 + lane * 16;
    const int hr = off / RB, hx = hr % HW_;
    const int u = ((off % RB) >> 4) ^ swz<RB>(hx);
    b_ok[j] = hr < HP;
    b_hy[j] = hr / HW_;
    b_hx[j] = hx;
    b_rel[j] = (b_hy[j] * W + hx) * (int)d.b_ps + rdn_coff32(d.b_c0 + c0 + u * 8, (int)d.b_ps, (int)d.b_pl);
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
    const unsigned st = __builtin_amdgcn_readfirstlane(lds_addr(lds) + stage * G_::STAGE);
#pragma unroll
    for (int j = 0; j < G_::PA; ++j) {
      const bool ok = a_ok[j] & (full | ((y0 + a_py[j] < H) & (x0 + a_px[j] < W)));
      glds16(ok ? (const void*)(ab + a_rel[j]) : (const void*)zero, st + (wave + NW * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < G_::PB; ++j) {
      const bool ok = b_ok[j] & (interior | (((unsigned)(y0 - 1 + b_hy[j]) < (unsigned)H) &
                                             ((unsigned)(x0 - 1 + b_hx[j]) < (unsigned)W)));
      glds16(ok ? (const void*)(hb + b_rel[j]) : (const void*)zero, st + (G_::A_PIECES + wave + NW * j) * 1024);
    }
  };

  // ---- per-lane fragment addresses (stage-relative; + immediates per k-step)
  const int xa = 4 * g + q;                               // pixel column of this lane's k rows
  int aoff[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
    aoff[i] = xa * RA + (((wm * (BM / G_::WMv) / 8 + 2 * i + (pp >> 1)) ^ swz<RA>(xa)) << 4) + (pp & 1) * 8;
  int boff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wn + G_::WNv * j;
    const int c = nt * 16 + 4 * pp;
    const int tp = c / CK, ci = c - tp * CK;
    const int ky = tp / 3, kx = tp - 3 * ky;
    const int hx = xa + kx;
    boff[j] = G_::A_PIECES * 1024 + (ky * HW_ + hx) * RB + (((ci >> 3) ^ swz<RB>(hx)) << 4) + (ci & 7) * 2;
  }

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const unsigned char* const st = lds + stage * G_::STAGE;
#pragma unroll
    for (int ks = 0; ks < TP / 32; ++ks) {
      bf16x8 af[MTW];
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const unsigned char* a = st + aoff[i] + ks * 32 * RA;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, a));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, a + 16 * RA));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const unsigned char* b = st + boff[j] + ks * 2 * HW_ * RB;
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(RDN_LDS_PTR(i16x4, b + HW_ * RB));
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int i = 0; i < MTW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
      }
    }
  };

  // ---- NS-deep ring: tiles it+1, it+2 in flight while tile it is multiplied;
  // unrolled by NS so that every stage offset is a constant
  static_assert(NS == 3, "wait counts below assume a 3-stage ring");
  if (t_cnt > 0) issue(t_beg, 0);
  if (t_cnt > 1) issue(t_beg + 1, 1);
  auto step = [&](int it, auto S) {
    constexpr int s = decltype(S)::value;
    if (it + 1 < t_cnt) wait_vm<G_::G>();   // own DMAs of tile it landed (tile it+1 may still fly)
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();           // everyone's landed; everyone done reading tile it-1's stage
    asm volatile("" ::: "memory");
    if (it + 2 < t_cnt) issue(t_beg + it + 2, (s + 2) % NS);
    compute(s);
  };
  for (int it = 0; it < t_cnt; it += NS) {
    step(it, std::integral_constant<int, 0>{});
    if (it + 1 < t_cnt) step(it + 1, std::integral_constant<int, 1>{});
    if (it + 2 < t_cnt) step(it + 2, std::integral_constant<int, 2>{});
  }

  // D[m][n]: row = g*4 + e (output channel), col = li (tile column)
  const int ncol_all = 9 * d.ndim;
  float* __restrict__ ws = d.ws + (int64_t)bz * d.mdim * ncol_all;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wn + G_::WNv * j;
    const int c = nt * 16 + li;
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
  RDN_PROBE("wgrad3_glds_kernel<bf16,%d,%d>", BM, CK);
  wgrad3_glds_kernel<BM, CK, 3><<<blocks, 256, 0, st>>>(*d, tiles_x, tiles_y, ntiles, tpb);
  return rdn_check_launch("rdn_conv_wgrad(conv3 glds)");
}

}  // namespace

// Tile shape of the LDS-DMA weight-gradient kernel for d, or 0 when it does not
// apply (fp32, a fused PReLU gate on operand A, channel counts off the grid).
int rdn_wgrad3_glds_pick(const rdn_wgrad_desc* d, int* bm, int* ck) {
  static const bool off = [] {
    const char* e = getenv("RDN_WGLDS");
    return e && e[0] == '0';
  }();
  if (off || d->dtype != RDN_BF16 || d->a_gate || d->mdim < 32 || d->ndim % 32) return 0;
  *bm = d->mdim <= 32 ? 32 : 64;
  *ck = d->ndim % 64 == 0 ? 64 : 32;
  return 1;
}

int rdn_wgrad3_glds_launch(const rdn_wgrad_desc* d, int bm, int ck, int blocks, int tiles_x, int tiles_y, int ntiles,
                           int tpb, hipStream_t st) {
  if (bm == 32) return ck == 64 ? launch<32, 64>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st)
                                : launch<32, 32>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
  if (bm == 64) return ck == 64 ? launch<64, 64>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st)
                                : launch<64, 32>(d, blocks, tiles_x, tiles_y, ntiles, tpb, st);
  rdn_set_error("rdn_conv_wgrad(conv3 glds): BM=%d CK=%d", bm, ck);
  return RDN_E_SHAPE;
}
