// 3x3 / pad 1 / stride 1 convolution as an implicit GEMM on large tiles (gfx950,
// bf16 MFMA): the MFMA-heavy convolutions of levels 1-3 in forward
// (Unet_model.py:72-89 dense convs, :35-43 up convs) and their input gradients (the
// same conv over dYpre with rotated, transposed weights; PReLU-backward gate
// optionally fused into the halo loader, as conv3_halo).
//
// Why a second halo kernel: conv3_halo (4 waves, 8 x 16 pixels x <= 128 columns)
// re-streams the weights from L2 for every 128 pixels and meets a barrier every
// 16-32 MFMAs per wave; at levels 2/3 it ran at 0.25-0.3 of the MFMA peak with
// 44 % of its wave cycles parked at waits.  Here:
//
// * block = 512 threads (8 waves, one block per CU) = a TH x 16 pixel tile (TH = 16:
//   256 pixels) x BN output columns; every weight byte staged in LDS feeds 256
//   pixels (half the L2 weight stream of the 128-pixel tile) and every wave owns a
//   64 x 64 (or 32 x 64 / 64 x 32) accumulator tile: 16 MFMAs per 8 fragment reads;
// * one LDS weight stage = TWO 64-deep K stages (256-B rows padded to 288 B:
//   conflict-free ds_read_b128), double buffered and register staged one stage
//   ahead, so a wave runs 32 MFMAs (64 x 64 tile) between two barriers;
// * the input halo [(TH+2) x 18][CK] of a channel chunk is loaded ONCE for all 9
//   taps, the next chunk's halo is prefetched into registers during the current
//   chunk;
// * MFMA operands are swapped (A = weights, B = pixels): a lane ends with four
//   consecutive output channels of one pixel, written to the fp32 epilogue tile in
//   LDS as one 16-byte store; the epilogue then applies bias / PReLU-input store /
//   PReLU / residual / accumulate as 16-byte NHWC units (conv3_halo's epilogue).
//
// Packed weights as for conv3_halo (rdn_pack_weights with ck > 0):
//   P[n][chunk*KC + tap*CK + ci],  KC = roundup(9*CK, 64).
#include "conv3_tile.h"

#include <cstdlib>
#include <utility>

namespace {

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>), unrolled
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int NTB = 512;
constexpr int TWB = 16;
constexpr int LDS_CAP = 160 * 1024;

template <int TH, int BN, int WM, int CK, bool GATE>
struct BigCfg {
  static constexpr int BM = TH * TWB;
  static constexpr int HWP = (TH + 2) * (TWB + 2);            // halo pixels
  static constexpr int HROW = c3::HaloRow<CK * 2>::V;         // bytes per halo pixel
  static constexpr int HALO_BYTES = (HWP * HROW + 15) / 16 * 16;
  static constexpr int KC = (9 * CK + 63) / 64 * 64;          // packed K per chunk
  static constexpr int SPC = KC / 64;                          // 64-deep K stages per chunk
  static constexpr int SS = (SPC + 1) / 2;                     // LDS stages (pairs) per chunk
  static constexpr int RW = 288;                               // LDS weight row: 2 x 128 B + 32 B pad
  static constexpr int W_BYTES = BN * RW;
  static constexpr int MAIN = HALO_BYTES + 2 * W_BYTES;
  static constexpr int CROW = BN * 4 + 16;                     // epilogue fp32 row (bytes)
  static constexpr int EPI = BM * CROW;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static constexpr int WN = 8 / WM;
  static constexpr int WTM = BM / WM, WTN = BN / WN;           // wave tile (pixels x columns)
  static constexpr int MT = WTM / 16, NTL = WTN / 16;
  static constexpr int HU = CK / 8;                            // 16-B units per halo pixel
  static constexpr int H_UNITS = HWP * HU;
  static constexpr int H_IT = (H_UNITS + NTB - 1) / NTB;
  static constexpr int B_UNITS = BN * 16;                      // 16-B weight units per LDS stage
  static constexpr int B_IT = (B_UNITS + NTB - 1) / NTB;
  static constexpr bool OK = LDS <= LDS_CAP && MT >= 1 && NTL >= 1 && WTM % 16 == 0 && WTN % 16 == 0 &&
                             (WTM / 16) * 16 == WTM && CK % 32 == 0 && (!GATE || NTB % HU == 0) &&
                             B_UNITS % NTB == 0;
};

template <int TH, int BN, int WM, int CK, bool GATE>
__global__ __launch_bounds__(NTB, 2) void conv3_big_kernel(rdn_conv_desc d, int tiles_x, int tiles_y) {
  using Cfg = BigCfg<TH, BN, WM, CK, GATE>;
  constexpr int VEC = 8;
  constexpr int BM = Cfg::BM, HROW = Cfg::HROW, RW = Cfg::RW, SPC = Cfg::SPC, SS = Cfg::SS;
  constexpr int WN = Cfg::WN, WTM = Cfg::WTM, WTN = Cfg::WTN, MT = Cfg::MT, NTL = Cfg::NTL;
  constexpr int HU = Cfg::HU, H_UNITS = Cfg::H_UNITS, H_IT = Cfg::H_IT, B_IT = Cfg::B_IT;
  constexpr int RS = TWB + 2;                                  // halo pixels per halo row
  static_assert(Cfg::OK, "conv3_big geometry");

  __shared__ __attribute__((aligned(16))) unsigned char lds[Cfg::LDS];
  unsigned char* const halo = lds;
  unsigned char* const wst = lds + Cfg::HALO_BYTES;            // two weight stages of BN x RW

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int r = lane & 15, g = lane >> 4;
  // 1-D grid, column tile fastest: the blocks reading one halo share an XCD
  const int ncb = (d.ncols + BN - 1) / BN;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  int bt = lb / ncb;
  const int tx = bt % tiles_x;
  bt /= tiles_x;
  const int ty = bt % tiles_y;
  const int nimg = bt / tiles_y;
  const int y0 = ty * TH, x0 = tx * TWB;
  const int n0 = (lb - (lb / ncb) * ncb) * BN;
  const int H = d.h, W = d.w;
  const int nch = d.cin / CK;

  // ---- halo units of this thread: element offset from the halo origin, LDS offset,
  // in-image flag; chunk c adds c * CK channels
  const int64_t hpix0 = ((int64_t)nimg * H + (y0 - 1)) * W + (x0 - 1);
  const bf16* const xb = (const bf16*)d.x + hpix0 * d.x_ps;
  const bf16* const gb = GATE ? (const bf16*)d.gate + hpix0 * d.gate_ps : nullptr;
  int hrel[H_IT], grel[GATE ? H_IT : 1], hlds[H_IT];
  bool hok[H_IT];
  const int hcu = (tid % HU) * VEC;   // NTB % HU == 0 for every CK used: fixed channel unit per thread
#pragma unroll
  for (int it = 0; it < H_IT; ++it) {
    const int u = tid + it * NTB;
    const int hp = u / HU;
    const int hy = hp / RS, hx = hp - hy * RS;
    hok[it] = u < H_UNITS && (unsigned)(y0 - 1 + hy) < (unsigned)H && (unsigned)(x0 - 1 + hx) < (unsigned)W;
    hrel[it] = (hy * W + hx) * (int)d.x_ps;
    if constexpr (GATE) grel[it] = (hy * W + hx) * (int)d.gate_ps;
    hlds[it] = u < H_UNITS ? hp * HROW + (u % HU) * 16 : -1;
  }
  u32x4 hreg[H_IT];
  u32x4 greg[GATE ? H_IT : 1];
  float galpha[GATE ? VEC : 1];
  auto load_halo = [&](int c) {
    const int64_t co = rdn_coff(d.x_c0 + c * CK + hcu, d.x_ps, d.x_pl);
    const int64_t cg = GATE ? rdn_coff(c * CK + hcu, d.gate_ps, d.gate_pl) : 0;
    if constexpr (GATE) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) galpha[q] = d.gate_alpha[c * CK + hcu + q];
    }
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      u32x4 v = {0u, 0u, 0u, 0u}, gv = {0u, 0u, 0u, 0u};
      if (hok[it]) {
        v = *(const u32x4*)(xb + hrel[it] + co);
        if constexpr (GATE) gv = *(const u32x4*)(gb + grel[it] + cg);
      }
      hreg[it] = v;
      if constexpr (GATE) greg[it] = gv;
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      if (hlds[it] < 0) continue;
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

  // ---- weight stages: LDS stage (c, jj) holds K stages 2jj, 2jj+1 of chunk c, i.e.
  // 16 units (256 B) of every output column n0..n0+BN
  u32x4 wreg[B_IT];
  const int wu = tid & 15;
  const bf16* const wb = (const bf16*)d.wp + (int64_t)(n0 + (tid >> 4)) * d.kp + wu * VEC;
  auto load_w = [&](int c, int jj) {
    const bool hi_ok = 2 * jj + 1 < SPC || wu < 8;   // the odd stage past the chunk: not loaded
#pragma unroll
    for (int it = 0; it < B_IT; ++it)
      wreg[it] = hi_ok ? *(const u32x4*)(wb + (int64_t)it * (NTB / 16) * d.kp + c * Cfg::KC + jj * 128)
                       : u32x4{0u, 0u, 0u, 0u};
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int it = 0; it < B_IT; ++it)
      *(u32x4*)(wst + buf * Cfg::W_BYTES + ((tid >> 4) + it * (NTB / 16)) * RW + wu * 16) = wreg[it];
  };

  // ---- fragment addresses: per-lane bases + compile-time immediates
  const unsigned char* const pa = halo + ((wm * MT) * RS + r) * HROW + g * 16;   // pixel frag rows
  const int b_lane = (wn * WTN + r) * RW + g * 16;

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K stage j (64 deep) of the current chunk, from weight buffer pbs (+h*128 B)
  auto compute = [&](auto JJ, const unsigned char* pbs) {
    constexpr int jj = decltype(JJ)::value;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * jj + h;
      if (j >= SPC) break;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int k0 = j * 64 + ks * 32;
        if (k0 >= 9 * CK) break;               // padded K: zero weights, skipped
        const int tap = k0 / CK, ci = k0 - (k0 / CK) * CK;
        const int ao = ((tap / 3) * RS + tap % 3) * HROW + ci * 2;
        u32x4 af[MT], bfr[NTL];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = *(const u32x4*)(pa + ao + i * RS * HROW);
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) bfr[jn] = *(const u32x4*)(pbs + jn * 16 * RW + h * 128 + ks * 64);
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

  load_halo(0);
  load_w(0, 0);
  store_halo();
  store_w(0);
  __syncthreads();
  int buf = 0;
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (more) load_halo(c + 1);   // in flight during this chunk's stages
    auto stage = [&](auto JJ) {
      constexpr int jj = decltype(JJ)::value;
      const bool nxt = jj + 1 < SS || more;
      if (nxt) load_w(jj + 1 < SS ? c : c + 1, jj + 1 < SS ? jj + 1 : 0);
      compute(JJ, wst + buf * Cfg::W_BYTES + b_lane);
      if (nxt) store_w(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    };
    static_for<SS>(stage);
    if (more) {
      store_halo();
      __syncthreads();
    }
  }

  // ---- epilogue: fp32 tile [BM pixels][BN columns] through LDS, then 16-B NHWC units
  constexpr int CROW = Cfg::CROW;
  {
    unsigned char* const ct = lds;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) {
        const int p = (wm * MT + i) * 16 + r;
        const int c = wn * WTN + jn * 16 + g * 4;
        *(f32x4*)(ct + p * CROW + c * 4) = acc[i][jn];
      }
  }
  __syncthreads();
  const float* const Ct = (const float*)lds;
  const int flags = d.flags;
  const bool fast = (d.ncols % VEC) == 0 && !(flags & RDN_EPI_OUT_NCHW) && y0 + TH <= H && x0 + TWB <= W &&
                    (!(flags & RDN_EPI_RESID) || (d.res_climit % VEC == 0 && d.res_ps % VEC == 0 &&
                                                  d.res_c0 % VEC == 0)) &&
                    d.out_ps % VEC == 0 && d.out_c0 % VEC == 0 && d.pre_ps % VEC == 0;
  if (!fast) {
    c3::store_tile<bf16, BN, NTB>(d, Ct, CROW / 4, y0, x0, nimg, n0, tid);
    return;
  }
  constexpr int UPR = BN / VEC, EU = BM * UPR, E_IT = (EU + NTB - 1) / NTB;
  constexpr bool COLFIX = NTB % UPR == 0;   // a thread's output channels are fixed
  const int64_t opix0 = ((int64_t)nimg * H + y0) * W + x0;
  float ebias[VEC], ealpha[VEC];
  int64_t cf_pre = 0, cf_out = 0, cf_res = 0;
  auto col_consts = [&](int c) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      ebias[q] = (flags & RDN_EPI_BIAS) ? d.bias[c + q] : 0.f;
      ealpha[q] = (flags & RDN_EPI_PRELU) ? d.alpha[c + q] : 0.f;
    }
    cf_pre = rdn_coff(c, d.pre_ps, d.pre_pl);
    cf_out = rdn_coff(d.out_c0 + c, d.out_ps, d.out_pl);
    cf_res = rdn_coff(d.res_c0 + c, d.res_ps, d.res_pl);
  };
  if constexpr (COLFIX) col_consts(n0 + (tid % UPR) * VEC);
#pragma unroll
  for (int it = 0; it < E_IT; ++it) {
    const int u = tid + it * NTB;
    if (EU % NTB && u >= EU) break;
    const int px = u / UPR, cl = (u - px * UPR) * VEC, c = n0 + cl;
    if constexpr (!COLFIX) col_consts(c);
    float v[VEC];
    const float* src = Ct + (px * CROW) / 4 + cl;
    const f32x4 t0 = *(const f32x4*)src, t1 = *(const f32x4*)(src + 4);
    v[0] = t0[0]; v[1] = t0[1]; v[2] = t0[2]; v[3] = t0[3];
    v[4] = t1[0]; v[5] = t1[1]; v[6] = t1[2]; v[7] = t1[3];
    const int64_t opix = opix0 + (px / TWB) * W + px % TWB;
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] += ebias[q];
    if (flags & RDN_EPI_STORE_PRE) *(u32x4*)((bf16*)d.pre + opix * d.pre_ps + cf_pre) = Unit16<bf16>::pack(v);
    if (flags & RDN_EPI_PRELU) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] = v[q] > 0.f ? v[q] : ealpha[q] * v[q];
    }
    bf16* const op = (bf16*)d.out + opix * d.out_ps + cf_out;
    float rv[VEC];
    if ((flags & RDN_EPI_RESID) && c < d.res_climit) {
      Unit16<bf16>::unpack(*(const u32x4*)((const bf16*)d.res + opix * d.res_ps + cf_res), rv);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += rv[q];
    }
    if (flags & RDN_EPI_ACCUM) {
      Unit16<bf16>::unpack(*(const u32x4*)op, rv);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += rv[q];
    }
    *(u32x4*)op = Unit16<bf16>::pack(v);
  }
}

int big_mode() {
  // RDN_BIG: unset/"1" = the default shape rule below; "0" = never (conv3_halo);
  // "all" = every bf16 shape the kernel can take (experiments)
  static const int m = [] {
    const char* e = getenv("RDN_BIG");
    if (!e) return 1;
    if (e[0] == '0') return 0;
    if (e[0] == 'a') return 2;
    return 1;
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

template <int TH, int BN, int WM, int CK>
int launch_big(const rdn_conv_desc* d, hipStream_t st) {
  constexpr bool OKP = BigCfg<TH, BN, WM, CK, false>::OK, OKG = BigCfg<TH, BN, WM, CK, true>::OK;
  const int tiles_x = (d->w + TWB - 1) / TWB, tiles_y = (d->h + TH - 1) / TH;
  const int64_t blocks = (int64_t)d->n * tiles_x * tiles_y * ((d->ncols + BN - 1) / BN);
  if (blocks >= (1ll << 31)) return 1;
  if (d->gate) {
    if constexpr (OKG) {
      RDN_PROBE("conv3_big_kernel<bf16,%d,%d,%d,%d,gate>", TH, BN, WM, CK);
      conv3_big_kernel<TH, BN, WM, CK, true><<<dim3((unsigned)blocks), NTB, 0, st>>>(*d, tiles_x, tiles_y);
      return rdn_check_launch("rdn_conv_fwd(conv3 big)");
    }
    return 1;
  }
  if constexpr (OKP) {
    RDN_PROBE("conv3_big_kernel<bf16,%d,%d,%d,%d>", TH, BN, WM, CK);
    conv3_big_kernel<TH, BN, WM, CK, false><<<dim3((unsigned)blocks), NTB, 0, st>>>(*d, tiles_x, tiles_y);
    return rdn_check_launch("rdn_conv_fwd(conv3 big)");
  }
  return 1;
}

template <int TH, int BN, int WM, int CK, bool GATE>
int blocks_per_cu() {
  static const int n = [] {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, conv3_big_kernel<TH, BN, WM, CK, GATE>, NTB, 0) !=
            hipSuccess || v < 1)
      v = 1;
    return v;
  }();
  return n;
}

// Candidate tiles (TH x 16 pixels x BN columns, WM waves along the pixels) and a
// per-block efficiency weight (larger wave tiles: more MFMAs per fragment read)
struct Plan { int th, bn, wm; double eff; };
constexpr Plan kPlans[] = {{16, 128, 4, 1.0}, {16, 96, 4, 0.95}, {16, 64, 4, 0.85},
                           {8, 160, 4, 0.9}, {8, 128, 2, 0.85}, {8, 64, 2, 0.7}};
constexpr int kNPlans = sizeof(kPlans) / sizeof(kPlans[0]);

template <int I, int CK>
int launch_plan(const rdn_conv_desc* d, hipStream_t st) {
  constexpr Plan p = kPlans[I];
  return launch_big<p.th, p.bn, p.wm, CK>(d, st);
}

template <int I, int CK>
int plan_bpc(bool gate) {
  constexpr Plan p = kPlans[I];
  if constexpr (BigCfg<p.th, p.bn, p.wm, CK, true>::OK) {
    if (gate) return blocks_per_cu<p.th, p.bn, p.wm, CK, true>();
  }
  if constexpr (BigCfg<p.th, p.bn, p.wm, CK, false>::OK) {
    if (!gate) return blocks_per_cu<p.th, p.bn, p.wm, CK, false>();
  }
  return 0;   // not instantiable
}

template <int CK, int... I>
void fill_bpc(int* bpc, bool gate, std::integer_sequence<int, I...>) {
  ((bpc[I] = plan_bpc<I, CK>(gate)), ...);
}

// tile plan: the candidate minimising (rounds of blocks over the resident slots) x
// (per-block cost), exact column tiling only
template <int CK>
int big_dispatch(const rdn_conv_desc* d, hipStream_t st) {
  const int cus = cu_count();
  const bool gate = d->gate != nullptr;
  int bpc[kNPlans];
  fill_bpc<CK>(bpc, gate, std::make_integer_sequence<int, kNPlans>{});
  int best = -1;
  double best_t = 1e30;
  for (int i = 0; i < kNPlans; ++i) {
    const Plan& p = kPlans[i];
    if (!bpc[i] || d->ncols % p.bn) continue;
    const int64_t tiles = (int64_t)d->n * ((d->h + p.th - 1) / p.th) * ((d->w + TWB - 1) / TWB);
    const int64_t blocks = tiles * (d->ncols / p.bn);
    const int64_t slots = (int64_t)cus * bpc[i];
    const double rounds = (double)((blocks + slots - 1) / slots);
    const double per_block = (double)p.th * p.bn / (16.0 * 128.0) / p.eff / bpc[i];
    const double t = rounds * per_block;
    if (t < best_t - 1e-9) { best_t = t; best = i; }
  }
  switch (best) {
    case 0: return launch_plan<0, CK>(d, st);
    case 1: return launch_plan<1, CK>(d, st);
    case 2: return launch_plan<2, CK>(d, st);
    case 3: return launch_plan<3, CK>(d, st);
    case 4: return launch_plan<4, CK>(d, st);
    case 5: return launch_plan<5, CK>(d, st);
  }
  return 1;
}

}  // namespace

// Level 1-3 bf16 3x3 convs with enough columns and input channels for the large
// tile (else 1: the caller falls back to conv3_ws / conv3_halo)
int rdn_conv3_big_launch(const rdn_conv_desc* d, int ck, hipStream_t st) {
  const int mode = big_mode();
  if (!mode || d->dtype != RDN_BF16 || d->gather != RDN_G_CONV3) return 1;
  if (d->bn || d->bm) return 1;
  if (ck != 32 && ck != 64) return 1;
  if (d->gate && (d->gate_ps % 8 || ((uintptr_t)d->gate & 15) || !d->gate_alpha)) return 1;
  if (d->ncols % 32 || d->ncols < 64 || d->cin < 64) return 1;
  if (d->x_ps % 8 || d->x_c0 % 8 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15) || d->kp % 8) return 1;
  if (mode == 1) {
    // default rule: grids of at least one block per CU at the 16 x 16 x 128 tile
    // (levels 1-3 of the 256^2 train step and larger)
    const int64_t px = (int64_t)d->n * d->h * d->w;
    if (px < 8192) return 1;
  }
  // per-thread halo offsets in 32 bits
  if ((int64_t)18 * d->w * d->x_ps >= (1ll << 30) || (d->gate && (int64_t)18 * d->w * d->gate_ps >= (1ll << 30)))
    return 1;
  return ck == 64 ? big_dispatch<64>(d, st) : big_dispatch<32>(d, st);
}
