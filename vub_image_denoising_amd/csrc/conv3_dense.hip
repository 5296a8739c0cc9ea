// Fused forward of the first three convolutions of a level-0 DenoisingBlock
// (Unet_model.py:81-87, base_filters 32: x has 32 channels, each conv adds 16):
//
//   out_0 = PReLU(conv_0(x)),  out_1 = PReLU(conv_1([x, out_0])),
//   out_2 = PReLU(conv_2([x, out_0, out_1]))
//
// in ONE pass over HBM.  Unfused, the three launches read x three times, out_0 twice
// and out_1 once (144 channels per pixel) to produce 96 (out_k and its PReLU input);
// here every block reads its tile's x once (with a 3-pixel halo) and keeps out_0 and
// out_1 in LDS for the next conv: 32 channels in, the same 96 out.  The halo is
// recomputed by neighbouring tiles: conv_0 runs on the 12 x 20 pixels around an
// 8 x 16 tile, conv_1 on 10 x 18, conv_2 on the tile itself (1.5x the MFMAs, which
// these HBM-bound layers have to spare).
//
// Block = 8 waves (two per SIMD), persistent over XCD-local tiles, one per CU.  LDS:
// * C: one image of the tile's 14 x 22-pixel region, 64 channels per pixel row
//   (x 0-31, out_0 32-47, out_1 48-63; 160-byte rows, see CP), so a K step of any of
//   the three convs addresses
//   "pixel + tap shift, channel" in one image (K is tap-major, channel-minor);
// * W2: conv_2's packed weights, resident (rdn_pack_weights with ck = cin; padded
//   rows, conflict-free); conv_0's and conv_1's are resident in registers instead
//   (each lane's A fragments for every k step: no weight reads per tile).  A first
//   form with all three panels in LDS and 4 waves ran 144 us for the three convs at
//   B16 (vs 118 us as three launches): one wave per SIMD left every LDS read exposed.
// MFMA operands are swapped (A = weights, B = pixels): a lane's accumulators are 4
// consecutive channels of one pixel, the 8-byte unit of the epilogue, which writes
// out_k (channel-blocked planes) and its PReLU input straight from the accumulators
// with buffer stores, only for the tile's own pixels; the next conv's copy in C is
// the same bf16 value the unfused path reads back from HBM, zero outside the image
// (the next conv's padding) -- results are bit-identical to three rdn_conv_fwd
// launches (tests/test_gpu_dense.py).  The next tile's x loads are in flight in
// registers while the current tile computes.
#include "rdn_common.h"

#include <cstdlib>
#include <cstring>

namespace {

constexpr int NW = 8, NT = 64 * NW;   // two waves per SIMD
// C row pitch (bytes): 128 + 32.  ds_read_b128 serves 64 lanes in four 16-lane groups
// that mix pixel rows r and k units g; checked over every k step and m-tile of the
// three convs, 144-B rows conflicted 2.6 / 2.6 / 2.0-way on average, 160-B rows
// 1.6 / 1.7 / 1.0 (the rest: output-region row breaks)
constexpr int CP = 160;

// Tile geometry (round 4: TH x TW = 16 x 32 where the image divides, else 8 x 16).
// The halo recompute per output pixel: conv_0 on (TH+4)(TW+4), conv_1 on (TH+2)(TW+2),
// in m-tiles of 16 region pixels padded to a multiple of the 8 waves: 4.0 MFMA
// slot-steps per pixel at 8 x 16, 3.06 at 16 x 32 (every B fragment is one LDS read:
// the convs' 16 output channels give each pixel fragment a single MFMA), and the x
// halo read 2.41 -> 1.63 times per pixel.
template <int TH_, int TW_>
struct DGeo {
  static constexpr int TH = TH_, TW = TW_;
  static constexpr int RW = TW + 6, RH = TH + 6;        // the x region (3-pixel halo)
  static constexpr int C_BYTES = RH * RW * CP;
  static constexpr int NXU = RH * RW * 4;               // 16-B units of x in the region
  static constexpr int X_IT = (NXU + NT - 1) / NT;
  static constexpr int mt(int npx) { return ((npx + 15) / 16 + NW - 1) / NW * NW; }
  static constexpr int NMT0 = mt((TH + 4) * (TW + 4)), NMT1 = mt((TH + 2) * (TW + 2)), NMT2 = mt(TH * TW);
};

template <int CIN> struct WCfg {
  static constexpr int K = 9 * CIN, NSTEP = (K + 31) / 32, KC = (K + 63) / 64 * 64;
  static constexpr int PITCH = KC * 2 + 32;     // conflict-free rows (every k step, 4 x 16-lane groups)
  static constexpr int BYTES = 16 * PITCH;
};
using W0 = WCfg<32>;
using W1 = WCfg<48>;
using W2 = WCfg<64>;

struct Out { __amdgpu_buffer_rsrc_t o, p; };

// LDS-only barrier: this wave's LDS writes retired, then s_barrier -- NOT
// __syncthreads(), whose vmcnt(0) would wait for the next tile's x loads and every
// epilogue store at each of the four barriers of a tile (the first form of this
// kernel: 115 us per launch without a single MFMA)
__device__ __forceinline__ void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// conv k (input channels CIN of C, output region halo HO: 2, 1, 0) over NMT m-tiles
// of 16 output-region pixels, MTW = NMT / NW per wave (m-tile wave + NW i); the
// weights are this lane's A fragments, resident in registers (wreg[j]: row r,
// k = 32 j + 8 g .. +7)
template <class G, int CIN, int HO, int NMT, bool WREG>
__device__ __forceinline__ void dense_conv(const unsigned char* __restrict__ lds, int wave, int r, int g,
                                           const u32x4* wreg, const unsigned char* __restrict__ wimg,
                                           f32x4 (&acc)[NMT / NW]) {
  constexpr int TH = G::TH, TW = G::TW, RW = G::RW;
  using WC = WCfg<CIN>;
  constexpr int MTW = NMT / NW;
  constexpr int OW = TW + 2 * HO;                      // output region width
  constexpr int NPX = (TH + 2 * HO) * OW;              // output region pixels
  constexpr int SH = 2 - HO;                           // output (oy, ox) -> C pixel (oy + SH + dy, ox + SH + dx)
  int pbase[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    int p = (wave + NW * i) * 16 + r;
    p = p < NPX ? p : NPX - 1;                         // padded lanes: a valid pixel, discarded
    const int oy = p / OW, ox = p - (p / OW) * OW;
    pbase[i] = ((oy + SH) * RW + ox + SH) * CP;
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < WC::NSTEP; ++j) {
    const int k = 32 * j + 8 * g;                      // this lane's 8 k: one tap, 8 channels
    int tap = k / CIN;
    const int ci = k - tap * CIN;
    tap = tap < 9 ? tap : 8;                           // padded k: zero weights, finite operand
    const int off = ((tap / 3) * RW + tap % 3) * CP + ci * 2;
    const u32x4 a = WREG ? wreg[j] : *(const u32x4*)(wimg + r * WC::PITCH + g * 16 + j * 64);
    u32x4 b[MTW];
#ifdef DN_DIAG_NO_LDS   // diagnostic build (timing only): opaque B fragments, no LDS reads
#pragma unroll
    for (int i = 0; i < MTW; ++i) asm volatile("" : "=v"(b[i]) : "v"(off));
#else
#pragma unroll
    for (int i = 0; i < MTW; ++i) b[i] = *(const u32x4*)(lds + pbase[i] + off);
#endif
#ifdef DN_DIAG_NO_MFMA
#pragma unroll
    for (int i = 0; i < MTW; ++i) { asm volatile("" ::"v"(a), "v"(b[i])); }
#else
#pragma unroll
    for (int i = 0; i < MTW; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b[i]),
                                                       acc[i], 0, 0, 0);
#endif
  }
}

// epilogue of conv k: bias, PReLU input (tile pixels), PReLU, output (tile pixels) and,
// for k < 2, the bf16 copy in C (channels 32 + 16k.., zero outside the image)
template <class G, int HO, int NMT, int KIDX>
__device__ __forceinline__ void dense_epi(unsigned char* __restrict__ lds, int wave, int r, int g, const f32x4 (&acc)[NMT / NW],
                                          const f32x4& bias, const f32x4& alpha, const Out& o, int y0, int x0, int H,
                                          int W) {
  constexpr int TH = G::TH, TW = G::TW, RW = G::RW;
  constexpr int MTW = NMT / NW;
  constexpr int OW = TW + 2 * HO;
  constexpr int NPX = (TH + 2 * HO) * OW;
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int p = (wave + NW * i) * 16 + r;
    const int oy = p / OW, ox = p - (p / OW) * OW;
    const int ty = oy - HO, tx = ox - HO;               // tile coordinates
    const bool live = p < NPX;
    const bool inimg = live && (unsigned)(y0 + ty) < (unsigned)H && (unsigned)(x0 + tx) < (unsigned)W;
    const bool own = live && (unsigned)ty < (unsigned)TH && (unsigned)tx < (unsigned)TW;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = acc[i][e] + bias[e];
    // tile pixel (ty, tx): element offset (ty * W + tx) * 16 + 4g from the tile origin
#ifdef DN_DIAG_NO_STORE
    int off = RDN_OOB;
#else
    int off = own ? ((ty * W + tx) * 16 + 4 * g) * 2 : RDN_OOB;
#endif
    asm volatile("" : "+v"(off));
    __builtin_amdgcn_raw_buffer_store_b64(rdn_pack4(v), o.p, off, 0, 0);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : alpha[e] * v[e];
    const u32x2 pk = rdn_pack4(v);
    __builtin_amdgcn_raw_buffer_store_b64(pk, o.o, off, 0, 0);
    if constexpr (KIDX < 2) {
      if (live)
        *(u32x2*)(lds + ((oy + 3 - HO) * RW + ox + 3 - HO) * CP + (32 + 16 * KIDX + 4 * g) * 2) =
            inimg ? pk : u32x2{0u, 0u};
    }
  }
}

template <int TH, int TW>
__global__ __launch_bounds__(NT, 1) void conv3_dense_kernel(rdn_dense3_desc d, int tiles_x, int tiles_y, int ntiles) {
  using G = DGeo<TH, TW>;
  constexpr int RW = G::RW, X_IT = G::X_IT, NXU = G::NXU;
  constexpr int W2_OFF = G::C_BYTES;              // conv_2's weights: LDS (registers: conv_0, conv_1)
  static_assert(W2_OFF + W2::BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char lds[W2_OFF + W2::BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int H = d.h, W = d.w;

  // tiles of this block: its XCD's contiguous share, strided by the XCD's block count
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7;
  const int t_hi = (int)((int64_t)ntiles * (xcd + 1) / 8);
  int t = (int)((int64_t)ntiles * xcd / 8) + (blockIdx.x >> 3);
  if (t >= t_hi) return;

  // ---- resident weights: every lane's A fragments of the three convs in registers
  // (the same for every tile: no LDS image, no per-k-step weight reads)
  // (conv_2's 18 k-steps as well spilled at 256 VGPRs: its panel stays in LDS)
  u32x4 w0[W0::NSTEP], w1[W1::NSTEP];
  auto load_w = [&](const bf16* wp, int kp, u32x4* wr, int nstep) {
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (j < nstep) wr[j] = *(const u32x4*)(wp + (int64_t)r * kp + 32 * j + 8 * g);
  };
  load_w((const bf16*)d.wp[0], d.kp[0], w0, W0::NSTEP);
  load_w((const bf16*)d.wp[1], d.kp[1], w1, W1::NSTEP);
  {
    const bf16* wp = (const bf16*)d.wp[2];
    for (int u = tid; u < 16 * (W2::KC / 8); u += NT) {
      const int n = u / (W2::KC / 8), k8 = u - n * (W2::KC / 8);
      *(u32x4*)(lds + W2_OFF + n * W2::PITCH + k8 * 16) = *(const u32x4*)(wp + (int64_t)n * d.kp[2] + k8 * 8);
    }
  }
  f32x4 bias[3], alpha[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bias[k][e] = d.bias[k][4 * g + e];
      alpha[k][e] = d.alpha[k][4 * g + e];
    }

  // ---- x region loads: unit u -> region pixel u / 4, x channels 8 (u % 4) ..; the
  // two 16-channel planes of the block buffer (channel-blocked, 32-byte pixel rows)
  // (unit it of this thread: recomputed per use -- four index arrays of X_IT registers
  // each spilled the 16 x 32 geometry)
  auto xunit = [&](int it, int& hy, int& hx, int& rel, int& lo) {
    const int u = tid + it * NT;
    const int hp = u < NXU ? u / 4 : 0, cu = u & 3;
    hy = hp / RW;
    hx = hp - hy * RW;
    rel = (cu >> 1) * (int)d.x_pl + (hy * W + hx) * 16 + (cu & 1) * 8;
    lo = u < NXU ? hp * CP + cu * 16 : -1;
  };
  u32x4 xr[X_IT];
  auto load_x = [&](int tt) {
    const int tx = tt % tiles_x, t1 = tt / tiles_x;
    const int y0 = (t1 % tiles_y) * TH, x0 = tx * TW, nimg = t1 / tiles_y;
    const __amdgpu_buffer_rsrc_t rx = rdn_rsrc((const bf16*)d.x + (((int64_t)nimg * H + (y0 - 3)) * W + (x0 - 3)) * 16);
#pragma unroll
    for (int it = 0; it < X_IT; ++it) {
      int hy, hx, rel, lo;
      xunit(it, hy, hx, rel, lo);
      const bool ok = lo >= 0 && (unsigned)(y0 - 3 + hy) < (unsigned)H && (unsigned)(x0 - 3 + hx) < (unsigned)W;
      xr[it] = rdn_ld16(rx, ok, rel * 2);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < X_IT; ++it) {
      int hy, hx, rel, lo;
      xunit(it, hy, hx, rel, lo);
      if (lo >= 0) *(u32x4*)(lds + lo) = xr[it];
    }
  };

  load_x(t);
  store_x();
  __syncthreads();
  while (t < t_hi) {
    const int nxt = t + per;
    const int tx = t % tiles_x, t1 = t / tiles_x;
    const int y0 = (t1 % tiles_y) * TH, x0 = tx * TW, nimg = t1 / tiles_y;
#ifndef DN_DIAG_NO_XLOAD   // diagnostic build (timing only): every tile computes on the first tile's x
    if (nxt < t_hi) load_x(nxt);   // in flight during this tile
#endif
    const int64_t pix0 = ((int64_t)nimg * H + y0) * W + x0;
    Out o[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      o[k].o = rdn_rsrc((const bf16*)d.out[k] + pix0 * 16);
      o[k].p = d.pre[k] ? rdn_rsrc((const bf16*)d.pre[k] + pix0 * 16) : rdn_rsrc_none(d.out[k]);   // (no PReLU input kept)
    }
    {
      f32x4 acc[G::NMT0 / NW];
      dense_conv<G, 32, 2, G::NMT0, true>(lds, wave, r, g, w0, nullptr, acc);
      dense_epi<G, 2, G::NMT0, 0>(lds, wave, r, g, acc, bias[0], alpha[0], o[0], y0, x0, H, W);
    }
#ifndef DN_DIAG_NO_BAR
    bar_lds();
#endif
    {
      f32x4 acc[G::NMT1 / NW];   // (8 x 16: 12 m-tiles padded to 16, the critical path either way)
      dense_conv<G, 48, 1, G::NMT1, true>(lds, wave, r, g, w1, nullptr, acc);
      dense_epi<G, 1, G::NMT1, 1>(lds, wave, r, g, acc, bias[1], alpha[1], o[1], y0, x0, H, W);
    }
#ifndef DN_DIAG_NO_BAR
    bar_lds();
#endif
    {
      f32x4 acc[G::NMT2 / NW];
      dense_conv<G, 64, 0, G::NMT2, false>(lds, wave, r, g, nullptr, lds + W2_OFF, acc);
      dense_epi<G, 0, G::NMT2, 2>(lds, wave, r, g, acc, bias[2], alpha[2], o[2], y0, x0, H, W);
    }
    bar_lds();   // C's x rows are free (the compiler's own vmcnt wait before store_x
                 // counts the epilogue stores issued after the x loads)
#ifndef DN_DIAG_NO_XLOAD
    if (nxt < t_hi) {
      store_x();
      bar_lds();
    }
#endif
    t = nxt;
  }
}

// tile geometry: RDN_DENSE_TILE = 8x16 (round 3) | 16x16 | 8x32 (read per launch: the
// GPU test runs every geometry); 16 x 32 spilled 156 B/lane at 256 VGPRs
int dense_tile() {
  const char* e = getenv("RDN_DENSE_TILE");
  if (e && !strcmp(e, "8x16")) return 0;
  if (e && !strcmp(e, "16x16")) return 1;
  return 2;
}

template <int TH, int TW>
int launch_dense(const rdn_dense3_desc* d, hipStream_t st) {
  const int tiles_x = d->w / TW, tiles_y = d->h / TH;
  const int64_t ntiles = (int64_t)d->n * tiles_x * tiles_y;
  if (ntiles >= (1ll << 31)) { rdn_set_error("rdn_dense3_fwd: too many tiles"); return RDN_E_SHAPE; }
  // 32-bit buffer offsets from a tile's origin (x: plane 1 + 3-pixel halo rows)
  if (2 * (d->x_pl + (int64_t)(TH + 7) * d->w * 16) >= (int64_t)RDN_OOB - 64) {
    rdn_set_error("rdn_dense3_fwd: planes too far apart for 32-bit offsets");
    return RDN_E_SHAPE;
  }
  RDN_PROBE("conv3_dense_kernel<bf16,32,16,%dx%d>", TH, TW);
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8) cus = 256;
  int64_t per_xcd = (ntiles + 7) / 8;
  int slots = cus / 8;
  if (slots > per_xcd) slots = (int)per_xcd;
  conv3_dense_kernel<TH, TW><<<8 * slots, NT, 0, st>>>(*d, tiles_x, tiles_y, (int)ntiles);
  return rdn_check_launch("rdn_dense3_fwd");
}

}  // namespace

extern "C" int rdn_dense3_fwd(const rdn_dense3_desc* d, void* stream) {
  if (!d || !d->x) { rdn_set_error("rdn_dense3_fwd: null descriptor"); return RDN_E_ARG; }
  for (int k = 0; k < 3; ++k)
    if (!d->out[k] || !d->wp[k] || !d->bias[k] || !d->alpha[k] ||
        ((uintptr_t)d->out[k] & 15) || ((uintptr_t)d->pre[k] & 15) || ((uintptr_t)d->wp[k] & 15) || d->kp[k] % 8) {
      rdn_set_error("rdn_dense3_fwd: conv %d: null or unaligned operand", k);
      return RDN_E_ARG;
    }
  if (d->x_c == 64) return rdn_dense3_l1_launch(d, (hipStream_t)stream);   // level 1 (conv3_dense1.hip)
  if (d->x_c != 0 && d->x_c != 32) {
    rdn_set_error("rdn_dense3_fwd: x_c %d (32: level 0, 64: level 1)", d->x_c);
    return RDN_E_ARG;
  }
  if (d->kp[0] < W0::KC || d->kp[1] < W1::KC || d->kp[2] < W2::KC) {
    rdn_set_error("rdn_dense3_fwd: packed K too small (pack with ck = cin)");
    return RDN_E_SHAPE;
  }
  if (d->n <= 0 || d->h % 8 || d->w % 16 || ((uintptr_t)d->x & 15) || d->x_pl < (int64_t)d->n * d->h * d->w * 16) {
    rdn_set_error("rdn_dense3_fwd: needs H %% 8 == 0, W %% 16 == 0 and a channel-blocked x (16-channel planes)");
    return RDN_E_SHAPE;
  }
  // (256-pixel tiles: at least one tile per CU, else the 8 x 16 grid fills the chip better)
  const int tile = dense_tile();
  const int64_t px = (int64_t)d->n * d->h * d->w;
  if (tile == 1 && d->h % 16 == 0 && d->w % 16 == 0 && px >= 256ll * 256)
    return launch_dense<16, 16>(d, (hipStream_t)stream);
  if (tile == 2 && d->w % 32 == 0 && px >= 256ll * 256)
    return launch_dense<8, 32>(d, (hipStream_t)stream);
  return launch_dense<8, 16>(d, (hipStream_t)stream);
}

// name of the instantiation (tile geometry) rdn_dense3_fwd would launch for d
extern "C" int rdn_dense3_kernel_name(const rdn_dense3_desc* d, char* buf, int32_t len) {
  if (!buf || len < 1) { rdn_set_error("rdn_dense3_kernel_name: no buffer"); return RDN_E_ARG; }
  buf[0] = 0;
  rdn_probe_buf = buf;
  rdn_probe_len = len;
  const int rc = rdn_dense3_fwd(d, nullptr);
  rdn_probe_buf = nullptr;
  return rc;
}
