// Fused forward of the first three convolutions of a level-1 DenoisingBlock
// (Unet_model.py:81-87 at base_filters 32: x has 64 channels, each conv adds 32):
//
//   out_0 = PReLU(conv_0(x)),  out_1 = PReLU(conv_1([x, out_0])),
//   out_2 = PReLU(conv_2([x, out_0, out_1]))
//
// in ONE pass over HBM (round 6; the level-0 form is conv3_dense.hip).  Unfused, the
// three launches read x three times and out_0 twice (288 channels per pixel) to write
// 192 (out_k and its PReLU input); here a block reads its 16 x 16 tile's x once, with
// a 3-pixel halo, and keeps out_0 / out_1 in LDS: 64 channels in, the same 192 out.
// The halo is recomputed by neighbouring tiles (conv_0 on 20 x 20 pixels, conv_1 on
// 18 x 18).  Unlike level 0, the convs are not HBM-bound once fused: 87 GFLOP per
// block at batch 32 (x 1.26 with the halo), so the kernel is laid out for the MFMA
// pipe and the LDS bandwidth that feeds it.
//
// Block = 8 waves (two per SIMD), persistent over XCD-local tiles, one per CU.
// MFMA v_mfma_f32_32x32x16_bf16 with A = weights (the 32 output channels) and B =
// 32 pixels: with only 32 output channels a pixel fragment feeds ONE MFMA, so the
// 32 x 32 instruction halves the LDS bytes per FLOP of the 16 x 16 one.  LDS:
// * X: the tile's 22 x 22 x region, 64 channels; pixel rows of 9 16-B slots (8 used)
//   and image rows of 212 slots (== 4 mod 16).  The region arrives by LDS-DMA
//   (global_load_lds_dwordx4 in 1-KB pieces, out-of-image pixels from a zero line),
//   issued for the next tile in conv_2's second half, once conv_2 has read its x part.
// * OUT: out_0 | out_1 (64 channels) on the 20 x 20 grid conv_0 produces, same slot
//   geometry (20 x 9 = 180 slots per row, == 4 mod 16), written by the epilogues.
// * a ring of three 8-KB weight chunks (32 rows x 128 k, 16-B unit u of row r at
//   u ^ (r & 15)): the packed weights (rdn_pack_weights CONV_FWD, chunked K order)
//   stream through it by LDS-DMA, two chunks ahead -- 166 KB of weights per tile do
//   not fit beside the image.  21 chunk steps per tile (5 + 7 + 9), one barrier each.
// Bank conflicts (exhaustive model of the ds_read_b128 lane groups): an m-tile is two
// 16-pixel row segments (the second one's columns rotated by 12) or, for the 4
// columns a 20- / 18-wide region leaves, 8 rows x 4 columns; with 9-slot pixels and
// 212 / 180-slot rows every B-fragment read of every tap is conflict-free, and the A
// reads from the ring are too.
// The epilogue (bias, PReLU-input store, PReLU, output store, and for conv_0 / conv_1
// the bf16 copy into OUT, zero outside the image) goes from the accumulators with
// v_permlane32_swap pairs into 16-B units.  Results match the three rdn_conv_fwd
// launches up to fp32 summation order (bf16-rounded out_0 / out_1 feed the next conv,
// as the HBM round trip does); tests/test_gpu_dense1.py.
#include "rdn_common.h"

#include <utility>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NW = 8, NT = 64 * NW;
constexpr int TH = 16, TW = 16;
constexpr int XR = TH + 6, XC = TW + 6;          // x region (3-pixel halo)
constexpr int XROW = 212;                        // 16-B slots per X row: 22 x 9 + 14 (== 4 mod 16)
constexpr int OGW = TW + 4;                      // OUT grid: the conv_0 region (x coords - 1)
constexpr int OROW = 180;                        // slots per OUT row: 20 x 9 (== 4 mod 16)
constexpr int X_PIECES = (XR * XROW * 16 + 1023) / 1024;   // 73 DMA pieces
constexpr int XPW = (X_PIECES + NW - 1) / NW;    // 10 per wave (the pad pieces go to a dump)
constexpr int OFF_X = 0;
constexpr int OFF_DUMP = X_PIECES * 1024;        // 74752
constexpr int OFF_OUT = OFF_DUMP + 1024;
constexpr int OFF_RING = OFF_OUT + (TH + 4) * OROW * 16;   // + 57600
constexpr int CHUNK = 8192;                      // 32 rows x 128 k x bf16
constexpr int OFF_BA = OFF_RING + 3 * CHUNK;     // bias / slopes of the three convs
constexpr int LDS_BYTES = OFF_BA + 6 * 32 * 4;
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

// the convs: K side 64 / 96 / 128 channels; k-steps of 16 (packed K order: conv_0 and
// conv_1 tap-major over all channels, conv_2 in two rdn_conv3 chunks: x then out_0|out_1)
constexpr int NSTEP[3] = {36, 54, 72};
constexpr int NCH[3] = {5, 7, 9};                // weight chunks of 8 k-steps
constexpr int CH0[3] = {0, 5, 12};               // first chunk step of each conv
constexpr int NSTEPS = 21;                       // chunk steps per tile
constexpr int SH[3] = {0, 1, 2};                 // output region origin in x coords - 1 ... (see bx)
constexpr int RW_[3] = {20, 18, 16};             // output region width / height
constexpr int NWIDE[3] = {10, 9, 8};             // two-row 16-pixel m-tiles
constexpr int NMT[3] = {13, 12, 8};              // + narrow 8 x 4 m-tiles (x0 16 / 14)
constexpr int NX0[3] = {16, 14, 0};

constexpr int conv_of(int c) { return c < 5 ? 0 : c < 12 ? 1 : 2; }
constexpr bool conv_end(int c) { return c == 4 || c == 11 || c == 20; }
// next tile's x DMA pieces issued in chunk step c (after conv_2 read its x part in
// step 16; all before step 19's weight DMA, which the next tile's first wait covers)
constexpr int xdma_n(int c) { return c == 17 ? 4 : (c == 18 || c == 19) ? 3 : 0; }
constexpr int xdma_first(int c) { return c == 17 ? 0 : c == 18 ? 4 : 7; }
constexpr int stores_n(int c) { return conv_end(c) ? 8 : 0; }   // epilogue stores per lane
constexpr int md(int c) { return (c % NSTEPS + NSTEPS) % NSTEPS; }
// vector-memory ops this wave issued after chunk c's DMA (issued in step c - 2) by the
// time step c waits for it: step c-2's stores, step c-1's x pieces, its weight DMA
// (chunk c + 1) and its stores
constexpr int vm_after(int c) { return stores_n(md(c - 2)) + xdma_n(md(c - 1)) + 1 + stores_n(md(c - 1)); }

__device__ __attribute__((aligned(64))) unsigned int g_dn1_zero[16];

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// one LDS-DMA wave-instruction: 16 B per lane from `src` to LDS byte dst + lane * 16
// (dst wave-uniform, in M0); not counted by the compiler: the explicit vmcnt waits are
// the ordering
__device__ __forceinline__ void glds16(const void* src, unsigned dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}
// opaque copy: keeps loop-invariant address arithmetic inside the tile loop (hoisted,
// the 21 chunk DMAs' and the epilogues' invariants spilled 328 B/lane)
__device__ __forceinline__ int opq(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ unsigned lds_addr(const unsigned char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

// output-region pixel (y, x) of lane j (0..31) in m-tile m of conv k
template <int K>
__device__ __forceinline__ void mt_pixel(int m, int j, int& y, int& x) {
  if (m < NWIDE[K]) {
    y = 2 * m + (j >> 4);
    x = j < 16 ? j : ((j - 4) & 15);   // second segment rotated: (j - 16 + 12) & 15
  } else {
    y = 8 * (m - NWIDE[K]) + (j >> 2);
    x = NX0[K] + (j & 3);
    y = y < RW_[K] ? y : RW_[K] - 1;   // (rows past the region: a duplicate, discarded)
  }
}

template <class F, int... C>
__device__ __forceinline__ void for_steps(F&& f, std::integer_sequence<int, C...>) {
  (f(std::integral_constant<int, C>{}), ...);
}

struct Tile {
  int n, y0, x0;
};

struct Args {
  const bf16* x;
  int64_t x_pl;
  bf16* out[3];
  bf16* pre[3];
  const bf16* wp[3];
  int kp[3];
};

__global__ __launch_bounds__(NT, 1) void conv3_dense1_kernel(rdn_dense3_desc d, int tiles_x, int tiles_y, int ntiles) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j32 = lane & 31, h = lane >> 5;
  const int H = d.h, W = d.w;

  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7;
  const int t_lo = (int)((int64_t)ntiles * xcd / 8), t_hi = (int)((int64_t)ntiles * (xcd + 1) / 8);
  int t = t_lo + (blockIdx.x >> 3);
  if (t >= t_hi) return;
  const int t_last = t_hi - 1;

  const bf16* const X = (const bf16*)d.x;
  float* const bal = (float*)(lds + OFF_BA);
  if (tid < 64) {   // [conv][bias | alpha][32] (constant conv index: no dynamic kernel-argument indexing)
    const int c = tid & 31, ab = tid >> 5;
    bal[0 * 64 + tid] = ab ? d.alpha[0][c] : d.bias[0][c];
    bal[1 * 64 + tid] = ab ? d.alpha[1][c] : d.bias[1][c];
    bal[2 * 64 + tid] = ab ? d.alpha[2][c] : d.bias[2][c];
  }

  auto tile_of = [&](int tt) {
    Tile q;
    const int tx = tt % tiles_x;
    tt /= tiles_x;
    q.y0 = (tt % tiles_y) * TH;
    q.x0 = tx * TW;
    q.n = tt / tiles_y;
    return q;
  };

  // ---- x region DMA: piece pc = wave + 8 i (1 KB) of a tile; slot S = 64 pc + lane -> row
  // S / XROW, pixel (S % XROW) / 9, unit (S % XROW) % 9 (unit 8 and the row pad: zero
  // line).  The per-lane geometry is tile-invariant and computed once (the per-piece
  // divisions and 64-bit address arithmetic were ~50 VALU per piece and tile): the source
  // offset from the region origin (-1: a pad slot) and the region pixel ry << 8 | rx.
  int xrel[XPW], xyx[XPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int pc = wave + NW * i, S = pc * 64 + lane;
    const int ry = S / XROW, rem = S - ry * XROW, rx = rem / 9, u = rem - rx * 9;
    const bool ok = pc < X_PIECES && ry < XR && rx < XC && u < 8;
    xrel[i] = ok ? (u >> 2) * (int)d.x_pl + (ry * W + rx) * 32 + (u & 3) * 8 : -1;
    xyx[i] = ry << 8 | rx;
  }
  auto issue_x = [&](const Tile& q, int i) {
    const int pc = wave + NW * i;   // wave-uniform
    const unsigned dst = pc < X_PIECES ? lds_addr(lds + OFF_X) + pc * 1024 : lds_addr(lds + OFF_DUMP);
    const bf16* const base = X + (((int64_t)q.n * H + q.y0 - 3) * W + q.x0 - 3) * 32;
    const bool interior = q.y0 >= 3 && q.y0 + TH + 3 <= H && q.x0 >= 3 && q.x0 + TW + 3 <= W;
    bool ok = xrel[i] >= 0;
    if (!interior)
      ok = ok && (unsigned)(q.y0 - 3 + (xyx[i] >> 8)) < (unsigned)H && (unsigned)(q.x0 - 3 + (xyx[i] & 255)) < (unsigned)W;
    glds16(ok ? (const void*)(base + xrel[i]) : (const void*)g_dn1_zero, dst);
  };
  // ---- weight chunk c (0..20) into ring slot c % 3: this wave's piece = rows 4w..4w+3
  const int wrow = 4 * wave + (lane >> 4);
  const int wpu = lane & 15;
  auto issue_w = [&](auto CC) {
    constexpr int c = decltype(CC)::value, k = conv_of(c), jj = c - CH0[k];
    const int u = wpu ^ (wrow & 15);
    const int col = opq(128 * jj + 8 * u);
    const void* src = col < d.kp[k] ? (const void*)((const bf16*)d.wp[k] + (int64_t)wrow * d.kp[k] + col)
                                    : (const void*)g_dn1_zero;
    glds16(src, lds_addr(lds + OFF_RING + (c % 3) * CHUNK) + wave * 1024);
  };

  // A-fragment byte offsets in a ring slot: row j32, unit (2 s + h) ^ (j32 & 15)
  int aoff[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) aoff[s] = j32 * 256 + 16 * ((2 * s + h) ^ (j32 & 15));

  // ---- prologue: tile t's x, chunks 0 and 1
#pragma unroll
  for (int i = 0; i < XPW; ++i) issue_x(tile_of(t), i);
  issue_w(std::integral_constant<int, 0>{});
  issue_w(std::integral_constant<int, 1>{});
  wait_vm<0>();
  __syncthreads();   // (also the bias / slope table)

  // slots of this wave per conv: m-tiles {w, w + 8} (conv_0 / conv_1), {w, w + 4} on
  // waves 0-3 (conv_2); per SIMD (waves w, w + 4) that is 4 / 3 / 2 m-tiles
  const int ns0 = wave + 8 < NMT[0] ? 2 : 1, ns1 = wave + 8 < NMT[1] ? 2 : 1, ns2 = wave < 4 ? 2 : 0;

  f32x16 acc[2];
  int bx[2], bo[2];   // per slot: X / OUT byte base of this lane's pixel (tap 0, unit h)

  auto conv_begin = [&](auto KC) {
    constexpr int K = decltype(KC)::value;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int m = K == 2 ? wave + 4 * sl : wave + 8 * sl;
      int y, x;
      mt_pixel<K>(m < NMT[K] ? m : 0, opq(j32), y, x);
      bx[sl] = ((y + SH[K]) * XROW + (x + SH[K]) * 9 + h) * 16;
      bo[sl] = ((y + SH[K] - 1) * OROW + (x + SH[K] - 1) * 9 + h) * 16;
      acc[sl] = (f32x16)(0.f);
    }
  };

  // k-step s of conv K: B operand byte offset from the slot base (compile time)
  auto bsrc = [](int K, int s, bool& from_out) -> int {
    int tap, cg;
    if (K == 0) { tap = s / 4; cg = s % 4; from_out = false; }
    else if (K == 1) { tap = s / 6; cg = s % 6; from_out = cg >= 4; if (from_out) cg -= 4; }
    else { from_out = s >= 36; const int s2 = from_out ? s - 36 : s; tap = s2 / 4; cg = s2 % 4; }
    const int dy = tap / 3, dx = tap % 3;
    return from_out ? (dy * OROW + dx * 9 + 2 * cg) * 16 : (dy * XROW + dx * 9 + 2 * cg) * 16;
  };

  // MFMAs of chunk step C for NS slots.  (Every fragment of the step read into
  // registers before its first MFMA, 232 VGPRs: 152 -> 162 us per launch at B32, not
  // kept -- the LDS latency is not what bounds this kernel)
  auto compute = [&](auto CC, auto NSC) {
    constexpr int C = decltype(CC)::value, NS = decltype(NSC)::value;
    constexpr int K = conv_of(C), J = C - CH0[K];
    constexpr int NK = NSTEP[K] - 8 * J < 8 ? NSTEP[K] - 8 * J : 8;
    const unsigned char* const ring = lds + OFF_RING + (C % 3) * CHUNK;
#pragma unroll
    for (int s8 = 0; s8 < NK; ++s8) {
      const int s = 8 * J + s8;
      bool fo = false;
      const int bofs = bsrc(K, s, fo);
#ifdef DN1_DIAG_NO_LDSRD   // diagnostic build (scripts/dense_kbench.py l1): opaque operands
      u32x4 a, b[2];
      asm volatile("" : "=v"(a));
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) asm volatile("" : "=v"(b[sl]));
      (void)bofs;
#else
      const u32x4 a = *(const u32x4*)(ring + aoff[s8]);
      u32x4 b[2];
#pragma unroll
      for (int sl = 0; sl < NS; ++sl)
        b[sl] = *(const u32x4*)(lds + (fo ? OFF_OUT + bo[sl] : OFF_X + bx[sl]) + bofs);
#endif
#ifdef DN1_DIAG_NO_MFMA   // diagnostic build: operands consumed without MFMAs
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) asm volatile("" ::"v"(a), "v"(b[sl]));
#else
#pragma unroll
      for (int sl = 0; sl < NS; ++sl)
        acc[sl] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b[sl]),
                                                          acc[sl], 0, 0, 0);
#endif
    }
  };

  // epilogue geometry of conv K's two slots (tile-invariant, computed once): the global
  // byte offset of the lane's 16-B unit in the tile (RDN_OOB: halo pixel or no m-tile),
  // the OUT-grid LDS byte offset of its unit for the next conv (conv_0 / conv_1; -1: no
  // m-tile) and its tile pixel (ty + 8) << 8 | (tx + 8) for the in-image test of
  // border tiles
  int eo[3][2], el[2][2], eyx[3][2];
  auto epi_geo = [&](auto KC) {
    constexpr int K = decltype(KC)::value;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int m = K == 2 ? wave + 4 * sl : wave + 8 * sl;
      const bool live = K == 2 ? (wave < 4) : (m < NMT[K]);
      int y, x;
      mt_pixel<K>(live ? m : 0, j32, y, x);
      const int ty = y - (2 - SH[K]), tx = x - (2 - SH[K]);   // tile coordinates
      const bool own = live && (unsigned)ty < (unsigned)TH && (unsigned)tx < (unsigned)TW;
      eo[K][sl] = own ? ((ty * W + tx) * 32 + 8 * h) * 2 : RDN_OOB;
      eyx[K][sl] = (ty + 8) << 8 | (tx + 8);
      if constexpr (K < 2)   // OUT coords of conv K's output pixel: (y + SH, x + SH)
        el[K][sl] = live ? ((y + SH[K]) * OROW + (x + SH[K]) * 9 + 4 * K + h) * 16 : -1;
    }
  };
  epi_geo(std::integral_constant<int, 0>{});
  epi_geo(std::integral_constant<int, 1>{});
  epi_geo(std::integral_constant<int, 2>{});

  // epilogue of conv K for tile q: every lane issues 8 stores (2 slots x {pre, out} x 2
  // units; slots without an m-tile and pixels outside the tile store at the OOB offset).
  // Bias add and PReLU slope products as packed fp32 pairs, bf16 pairs by one
  // v_cvt_pk_bf16_f32 each (the same rounding as the per-element casts)
  auto epilogue = [&](auto KC, const Tile& q) {
    constexpr int K = decltype(KC)::value;
    const int64_t pix0 = ((int64_t)q.n * H + q.y0) * W + q.x0;
    const __amdgpu_buffer_rsrc_t rp = d.pre[K] ? rdn_rsrc((const bf16*)d.pre[K] + pix0 * 32)
                                               : rdn_rsrc_none(d.out[K]);   // (forward-only: no PReLU input kept)
    const __amdgpu_buffer_rsrc_t ro = rdn_rsrc((const bf16*)d.out[K] + pix0 * 32);
    const bool border = q.y0 == 0 || q.x0 == 0 || q.y0 + TH >= H || q.x0 + TW >= W;
    const float* const bk = bal + K * 64;
    f32x4 bb[4], aa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // channels 8 i + 4 h .. + 3 (accumulator registers 4 i .. 4 i + 3)
      bb[i] = *(const f32x4*)(bk + 8 * i + 4 * h);
      aa[i] = *(const f32x4*)(bk + 32 + 8 * i + 4 * h);
    }
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      unsigned pk[8], ok[8];   // bf16 pairs: [2 i + e] = channels 8 i + 4 h + 2 e, + 1
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const f32x2 v = f32x2{acc[sl][4 * i + 2 * e], acc[sl][4 * i + 2 * e + 1]} + f32x2{bb[i][2 * e], bb[i][2 * e + 1]};
          const f32x2 av = v * f32x2{aa[i][2 * e], aa[i][2 * e + 1]};
          pk[2 * i + e] = rdn_cvt2(v[0], v[1]);
          ok[2 * i + e] = rdn_cvt2(v[0] > 0.f ? v[0] : av[0], v[1] > 0.f ? v[1] : av[1]);
        }
      // pairs of 4-channel groups (0, 1) and (2, 3) -> 16-B units: lanes < 32 hold channels
      // 16 P .. 16 P + 7, lanes >= 32 16 P + 8 .. + 15
#pragma unroll
      for (int P = 0; P < 2; ++P)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const auto sp = __builtin_amdgcn_permlane32_swap(pk[4 * P + e], pk[4 * P + 2 + e], false, false);
          pk[4 * P + e] = sp[0];
          pk[4 * P + 2 + e] = sp[1];
          const auto so = __builtin_amdgcn_permlane32_swap(ok[4 * P + e], ok[4 * P + 2 + e], false, false);
          ok[4 * P + e] = so[0];
          ok[4 * P + 2 + e] = so[1];
        }
      bool inimg = true;
      if (border)
        inimg = (unsigned)(q.y0 + (eyx[K][sl] >> 8) - 8) < (unsigned)H && (unsigned)(q.x0 + (eyx[K][sl] & 255) - 8) < (unsigned)W;
      const int off = eo[K][sl];
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        const u32x4 up = {pk[4 * P], pk[4 * P + 1], pk[4 * P + 2], pk[4 * P + 3]};
        const u32x4 uo = {ok[4 * P], ok[4 * P + 1], ok[4 * P + 2], ok[4 * P + 3]};
        const int o = off == RDN_OOB ? RDN_OOB : off + 32 * P;
#ifndef DN1_DIAG_NO_STORE   // diagnostic build: no global stores
        __builtin_amdgcn_raw_buffer_store_b128(up, rp, o, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(uo, ro, o, 0, 0);
#else
        asm volatile("" ::"v"(up), "v"(uo), "v"(o));
#endif
        if constexpr (K < 2) {   // the next conv's operand: OUT grid, units (out_K: 4 K) + 2 P + h
          if (el[K][sl] >= 0) {
            const u32x4 z = inimg ? uo : u32x4{0u, 0u, 0u, 0u};
            *(u32x4*)(lds + OFF_OUT + el[K][sl] + 32 * P) = z;
          }
        }
      }
    }
  };

  auto step = [&](auto CC, const Tile& q, const Tile& qn) {
    constexpr int C = decltype(CC)::value;
    constexpr int K = conv_of(C);
    wait_vm<vm_after(C)>();   // chunk C landed (this wave's piece)
#ifndef DN1_DIAG_NO_BAR       // diagnostic build (with NO_WDMA / NO_XDMA): no barriers
    bar_lds();                // every wave's piece; every wave done with step C - 1 (ring slot (C + 2) % 3)
#endif
#ifndef DN1_DIAG_NO_XDMA   // diagnostic build: every tile multiplies the first tile's x
    if constexpr (xdma_n(C) > 0) {
#pragma unroll
      for (int i = 0; i < xdma_n(C); ++i) issue_x(qn, xdma_first(C) + i);
    }
#endif
#ifndef DN1_DIAG_NO_WDMA   // diagnostic build: the ring keeps the prologue's chunks
    issue_w(std::integral_constant<int, (C + 2) % NSTEPS>{});
#endif
    if constexpr (C == CH0[K]) conv_begin(std::integral_constant<int, K>{});
    const int ns = K == 0 ? ns0 : K == 1 ? ns1 : ns2;
    if (ns == 2) compute(CC, std::integral_constant<int, 2>{});
    else if (ns == 1) compute(CC, std::integral_constant<int, 1>{});
    if constexpr (conv_end(C)) epilogue(std::integral_constant<int, K>{}, q);
  };

  for (;;) {
    const Tile q = tile_of(t);
    const Tile qn = tile_of(min(t + per, t_last));   // (past the range: a harmless re-load of this tile)
    for_steps([&](auto CC) { step(CC, q, qn); }, std::make_integer_sequence<int, NSTEPS>{});
    t += per;
    if (t >= t_hi) break;
  }
  wait_vm<0>();   // the DMAs issued for a tile past the range land before the LDS is released
}

}  // namespace

// level-1 form of rdn_dense3_fwd (d->x_c == 64), called from conv3_dense.hip
int rdn_dense3_l1_launch(const rdn_dense3_desc* d, hipStream_t st) {
  if (d->kp[0] < 576 || d->kp[1] < 896 || d->kp[2] < 1152 || d->kp[0] % 8 || d->kp[1] % 8 || d->kp[2] % 8) {
    rdn_set_error("rdn_dense3_fwd(level 1): packed K too small (kp %d %d %d)", d->kp[0], d->kp[1], d->kp[2]);
    return RDN_E_SHAPE;
  }
  if (d->n <= 0 || d->h % TH || d->w % TW || ((uintptr_t)d->x & 15) || d->x_pl % 8 || d->x_pl >= (1ll << 30) ||
      d->x_pl < (int64_t)d->n * d->h * d->w * 32) {
    rdn_set_error("rdn_dense3_fwd(level 1): needs H %% 16 == 0, W %% 16 == 0 and a channel-blocked x (32-channel planes)");
    return RDN_E_SHAPE;
  }
  const int tiles_x = d->w / TW, tiles_y = d->h / TH;
  const int64_t ntiles = (int64_t)d->n * tiles_x * tiles_y;
  if (ntiles >= (1ll << 31) || (int64_t)TH * d->w * 64 >= (1ll << 30)) {
    rdn_set_error("rdn_dense3_fwd(level 1): shape too large for 32-bit tile offsets");
    return RDN_E_SHAPE;
  }
  RDN_PROBE("conv3_dense1_kernel<bf16,64,32,16x16>");
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8) cus = 256;
  const int64_t per_xcd = (ntiles + 7) / 8;
  int slots = cus / 8;
  if (slots > per_xcd) slots = (int)per_xcd;
  conv3_dense1_kernel<<<8 * slots, NT, 0, st>>>(*d, tiles_x, tiles_y, (int)ntiles);
  return rdn_check_launch("rdn_dense3_fwd(level 1)");
}
