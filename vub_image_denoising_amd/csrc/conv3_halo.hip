// 3x3 / pad 1 / stride 1 convolution as an implicit GEMM with an LDS-resident
// input halo (gfx950, MFMA).  Serves every 3x3 conv of the network in forward
// (Unet_model.py:48-49,60-61,72-75,35) and their input gradients (the same conv
// over dYpre with 180-degree-rotated, transposed weights).
//
// Block = 256 threads (4 waves) = a TH x TW = 8 x 16 output-pixel tile of one
// image x BN output channels.  The input channels are walked in chunks of CK:
// a chunk's (TH+2) x (TW+2) halo tile is loaded ONCE into LDS and feeds all 9
// taps (the generic gather re-reads every input pixel 9x through L2).  The
// weights stream through a double-buffered LDS stage of 128 bytes per output
// channel (one tap of 64 bf16 / 32 fp32 channels, or several taps of a smaller
// chunk).  The next chunk's halo is prefetched into registers during the
// current chunk's 9 taps.  The epilogue stages the fp32 tile through LDS so
// every global store (PReLU input, output, residual read, accumulate read) is
// a 16-byte NHWC vector.
//
// Packed weight layout (rdn_pack_weights with ck > 0):
//   P[n][chunk*KC + tap*CK + ci],  KC = roundup(9*CK, SK),  SK = 128 B / elem.
#include "conv3_tile.h"

#include <cstdlib>

namespace {

constexpr int NT = 256;
using c3::TH;
using c3::TW;
using c3::BM;
using c3::HW_;
using c3::HaloRow;
constexpr int ROWB = 160;                  // B-stage row: 128 B + 32 B pad (conflict-free ds_read_b128)

// occupancy request: narrow tiles keep 2 waves/SIMD, wide tiles let the
// register allocator use up to 512 VGPRs (measured faster: scripts/kbench.py)
// SPLIT (rdn_conv_fwd_splitk): block row blockIdx.y walks input-channel chunks
// [y * c_per, (y + 1) * c_per) only and stores its raw fp32 tile to ws[y][pixel][ncols];
// conv_splitk_reduce_kernel sums the slices in a fixed order and applies the epilogue
template <typename T, int BN, int WMW, int CK, bool GATE, bool PAIR_OK, bool SPLIT = false>
__global__ __launch_bounds__(NT, (BN >= 64 ? 1 : 2)) void conv3_halo_kernel(rdn_conv_desc d, int tiles_x, int tiles_y,
                                                                          int c_per = 0, float* __restrict__ ws = nullptr) {
  constexpr int ES = sizeof(T);
  constexpr int VEC = TypeInfo<T>::VEC;
  constexpr int SK = 128 / ES;                       // k per stage
  constexpr int KSTEP = 4 * VEC;                     // k per MFMA step (4 lane groups x one 16-B unit)
  constexpr int CKB = CK * ES;                       // bytes per halo pixel row (data)
  constexpr int HROW = HaloRow<CKB>::V;
  constexpr int SPC = (9 * CK + SK - 1) / SK;        // stages per chunk
  constexpr int KC = SPC * SK;
  constexpr int WNW = 4 / WMW;
  constexpr int WTM = BM / WMW, WTN = BN / WNW;
  constexpr int MT = WTM / 16, NTL = WTN / 16;
  constexpr int HU = CK / VEC;                       // 16-B units per halo pixel
  constexpr int H_UNITS = HW_ * HU;
  constexpr int H_IT = (H_UNITS + NT - 1) / NT;
  constexpr int B_UNITS = BN * 8;
  constexpr int B_IT = (B_UNITS + NT - 1) / NT;
  constexpr int HALO_BYTES = HW_ * HROW;
  // PAIR: two consecutive 128-B K stages per LDS stage and barrier (bf16, <= 96
  // columns: two blocks per CU still fit); a 256-B row padded to 288 B keeps the
  // ds_read_b128 B fragments conflict-free.  The launcher takes it for grids of at
  // most two blocks per CU: there halving the barriers wins (level-2 forward -11 %,
  // level-1 -17 %), on larger grids the single-stage form's third resident block
  // per CU does (level-2/3 input gradients +10 % when paired)
  constexpr bool PAIR = PAIR_OK && ES == 2 && BN <= 96 && SPC >= 2;
  constexpr int RW = PAIR ? 288 : ROWB;              // LDS weight row of one (paired) stage
  constexpr int SS = PAIR ? (SPC + 1) / 2 : SPC;     // (paired) stages per chunk
  // WALL (split launches, <= 64 columns): a chunk's SPC weight stages are loaded at once
  // and held in LDS together -- a split block walks one or a few chunks, so the per-stage
  // load -> barrier chain of the double-buffered walk (9 dependent loads per fp32 chunk)
  // was its whole time
  constexpr bool WALL = SPLIT && !PAIR && BN <= 64 && HALO_BYTES + SPC * BN * RW <= 144 * 1024;
  constexpr int MAIN_BYTES = HALO_BYTES + (WALL ? SPC : 2) * BN * RW;
  constexpr int CROW = BN * 4 + 16;                  // epilogue fp32 tile row
  constexpr int EPI_BYTES = BM * CROW;
  constexpr int LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;   // (>= the 4 x 2 x BN gate-out partials)
  constexpr bool KALIGN = CK % KSTEP == 0;           // a k-step never straddles a tap
  constexpr int UPR = BN / VEC, EU = BM * UPR, E_IT = (EU + NT - 1) / NT;
  constexpr bool COLFIX = NT % UPR == 0;             // a thread's output channels are fixed
  static_assert(MT >= 1 && NTL >= 1 && (CK % VEC) == 0, "tile");
  static_assert(!GATE || NT % HU == 0, "fixed channel group per thread");

  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  unsigned char* const halo = lds;
  unsigned char* const bst = lds + HALO_BYTES;      // two weight stages of BN x RW

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WMW, wn = wave / WMW;
  const int r = lane & 15, g = lane >> 4;
  // 1-D grid, logical (column tile, pixel tile) with the column tile fastest: the
  // blocks reading one input halo share an XCD (xcd_remap)
  const int ncb = (d.ncols + BN - 1) / BN;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  int bt = lb / ncb;
  const int tx = bt % tiles_x; bt /= tiles_x;
  const int ty = bt % tiles_y;
  const int nimg = bt / tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;
  const int n0 = (lb - (lb / ncb) * ncb) * BN;
  const int H = d.h, W = d.w;
  const int c_lo = SPLIT ? (int)blockIdx.y * c_per : 0;
  const int nch = SPLIT ? min(d.cin / CK, c_lo + c_per) : d.cin / CK;

  // ---- halo units of this thread (tile fixed for the block): element offset
  // from the halo origin, LDS offset, in-image flag; chunk c adds c * CK
  const int64_t hpix0 = ((int64_t)nimg * H + (y0 - 1)) * W + (x0 - 1);
  const T* const xb = (const T*)d.x + hpix0 * d.x_ps;
  const T* const gb = GATE ? (const T*)d.gate + hpix0 * d.gate_ps : nullptr;
  int hrel[H_IT], grel[GATE ? H_IT : 1], hlds[H_IT], hcu[H_IT];
  bool hok[H_IT];
#pragma unroll
  for (int it = 0; it < H_IT; ++it) {
    const int u = tid + it * NT;
    const int hp = u / HU, cu = u - hp * HU;
    const int hy = hp / (TW + 2), hx = hp - hy * (TW + 2);
    hok[it] = u < H_UNITS && (unsigned)(y0 - 1 + hy) < (unsigned)H && (unsigned)(x0 - 1 + hx) < (unsigned)W;
    hrel[it] = (hy * W + hx) * (int)d.x_ps;
    if constexpr (GATE) grel[it] = (hy * W + hx) * (int)d.gate_ps;
    hcu[it] = cu * VEC;
    hlds[it] = u < H_UNITS ? hp * HROW + cu * 16 : -1;
  }
  u32x4 hreg[H_IT];
  u32x4 greg[GATE ? H_IT : 1];
  float galpha[GATE ? VEC : 1];
  auto load_halo = [&](int c) {
    if constexpr (GATE) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) galpha[q] = d.gate_alpha[c * CK + (tid % HU) * VEC + q];
    }
#pragma unroll
    for (int it = 0; it < H_IT; ++it) {
      u32x4 v = {0u, 0u, 0u, 0u}, gv = {0u, 0u, 0u, 0u};
      if (hok[it]) {
        // channel offset of this unit in chunk c (channel-blocked operands: rdn_coff)
        v = *(const u32x4*)(xb + hrel[it] + rdn_coff(d.x_c0 + c * CK + hcu[it], d.x_ps, d.x_pl));
        if constexpr (GATE) gv = *(const u32x4*)(gb + grel[it] + rdn_coff(c * CK + hcu[it], d.gate_ps, d.gate_pl));
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
        Unit16<T>::unpack(v, dy);
        Unit16<T>::unpack(greg[it], pr);
#pragma unroll
        for (int q = 0; q < VEC; ++q) dy[q] = pr[q] > 0.f ? dy[q] : galpha[q] * dy[q];
        v = Unit16<T>::pack(dy);
      }
      *(u32x4*)(halo + hlds[it]) = v;
    }
  };
  // ---- weight stages: 8 units (128 B) per output channel; stage (c, j) at c*KC + j*SK;
  // an LDS stage jj holds K stages PAIR ? {2jj, 2jj+1} : {jj}
  u32x4 breg[PAIR ? 2 : 1][B_IT];
  const int ku = tid & 7;
  const T* const wb = (const T*)d.wp + (int64_t)(n0 + (tid >> 3)) * d.kp + ku * VEC;
  auto load_b = [&](int c, int jj) {
#pragma unroll
    for (int h = 0; h < (PAIR ? 2 : 1); ++h) {
      const int j = PAIR ? 2 * jj + h : jj;
      if (j >= SPC) break;
#pragma unroll
      for (int it = 0; it < B_IT; ++it)
        if (tid + it * NT < B_UNITS) breg[h][it] = *(const u32x4*)(wb + (int64_t)it * (NT / 8) * d.kp + c * KC + j * SK);
    }
  };
  auto store_b = [&](int buf, int jj) {
#pragma unroll
    for (int h = 0; h < (PAIR ? 2 : 1); ++h) {
      if ((PAIR ? 2 * jj + h : jj) >= SPC) break;
#pragma unroll
      for (int it = 0; it < B_IT; ++it)
        if (tid + it * NT < B_UNITS)
          *(u32x4*)(bst + buf * (BN * RW) + ((tid >> 3) + it * (NT / 8)) * RW + h * 128 + ku * 16) = breg[h][it];
    }
  };

  // ---- fragment addresses: per-lane base + immediates
  const int a_lane = ((wm * (WTM / 16)) * (TW + 2) + r) * HROW;
  int offA[KALIGN ? 1 : 2 * SPC];
  if constexpr (!KALIGN) {
#pragma unroll
    for (int jk = 0; jk < 2 * SPC; ++jk) {
      const int k = jk * KSTEP + g * VEC;
      int tap = k / CK;
      const int ci = k - tap * CK;
      tap = tap < 9 ? tap : 8;   // padded k: zero weights, finite operand
      offA[jk] = a_lane + ((tap / 3) * (TW + 2) + tap % 3) * HROW + ci * ES;
    }
  }
  const unsigned char* const pa = halo + (KALIGN ? a_lane + g * 16 : 0);
  const int b_lane = (wn * WTN + r) * RW + g * 16;

  f32x4 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int j, const unsigned char* pbs) {   // stage j of the current chunk
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      int ao;
      if constexpr (KALIGN) {
        const int k0 = (2 * j + ks) * KSTEP;
        int tap = k0 / CK;
        const int ci = k0 - tap * CK;
        tap = tap < 9 ? tap : 8;
        ao = ((tap / 3) * (TW + 2) + tap % 3) * HROW + ci * ES;
      } else {
        ao = offA[2 * j + ks];
      }
      u32x4 af[MT], bfr[NTL];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *(const u32x4*)(pa + ao + i * (TW + 2) * HROW);
#pragma unroll
      for (int jn = 0; jn < NTL; ++jn) bfr[jn] = *(const u32x4*)(pbs + jn * 16 * RW + ks * 64);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < NTL; ++jn) {
          if constexpr (ES == 2) {
            acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                                 __builtin_bit_cast(bf16x8, bfr[jn]), acc[i][jn], 0, 0, 0);
          } else {
            const f32x4 a4 = __builtin_bit_cast(f32x4, af[i]);
            const f32x4 b4 = __builtin_bit_cast(f32x4, bfr[jn]);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], b4[e], acc[i][jn], 0, 0, 0);
          }
        }
    }
  };

  if constexpr (WALL) {
    u32x4 wall[SPC][B_IT];
    auto load_all = [&](int c) {
#pragma unroll
      for (int j = 0; j < SPC; ++j)
#pragma unroll
        for (int it = 0; it < B_IT; ++it)
          if (tid + it * NT < B_UNITS) wall[j][it] = *(const u32x4*)(wb + (int64_t)it * (NT / 8) * d.kp + c * KC + j * SK);
    };
    auto store_all = [&]() {
#pragma unroll
      for (int j = 0; j < SPC; ++j)
#pragma unroll
        for (int it = 0; it < B_IT; ++it)
          if (tid + it * NT < B_UNITS)
            *(u32x4*)(bst + j * (BN * RW) + ((tid >> 3) + it * (NT / 8)) * RW + ku * 16) = wall[j][it];
    };
    load_halo(c_lo);
    load_all(c_lo);
    store_halo();
    store_all();
    __syncthreads();
    for (int c = c_lo; c < nch; ++c) {
      const bool more = c + 1 < nch;
      if (more) {   // the next chunk's halo and weights in flight during this one's taps
        load_halo(c + 1);
        load_all(c + 1);
      }
#pragma unroll
      for (int j = 0; j < SPC; ++j) compute(j, bst + j * (BN * RW) + b_lane);
      if (more) {
        __syncthreads();
        store_halo();
        store_all();
      }
      __syncthreads();
    }
  }
  if constexpr (!WALL) {
  load_halo(c_lo);
  load_b(c_lo, 0);
  store_halo();
  store_b(0, 0);
  __syncthreads();
  int buf = 0;
  for (int c = c_lo; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (more) load_halo(c + 1);   // in flight during this chunk's stages
#pragma unroll
    for (int jj = 0; jj < SS; ++jj) {
      const bool nxt = jj + 1 < SS || more;
      if (nxt) load_b(jj + 1 < SS ? c : c + 1, jj + 1 < SS ? jj + 1 : 0);
      if constexpr (PAIR) {
        compute(2 * jj, bst + buf * (BN * RW) + b_lane);
        if (2 * jj + 1 < SPC) compute(2 * jj + 1, bst + buf * (BN * RW) + b_lane + 128);
      } else {
        compute(jj, bst + buf * (BN * RW) + b_lane);
      }
      if (nxt) store_b(buf ^ 1, jj + 1 < SS ? jj + 1 : 0);
      __syncthreads();
      buf ^= 1;
    }
    if (more) {
      store_halo();
      __syncthreads();
    }
  }
  }

  // ---- epilogue: fp32 tile through LDS, then 16-byte NHWC units
  const int flags = d.flags;
  const bool fast = (d.ncols % VEC) == 0 && !(flags & RDN_EPI_OUT_NCHW) && y0 + TH <= H && x0 + TW <= W &&
                    (!(flags & RDN_EPI_RESID) || (d.res_climit % VEC == 0 && d.res_ps % VEC == 0 &&
                                                  d.res_c0 % VEC == 0)) &&
                    d.out_ps % VEC == 0 && d.out_c0 % VEC == 0 && d.pre_ps % VEC == 0;
  const int64_t opix0 = ((int64_t)nimg * H + y0) * W + x0;
  // gate-out (d.gout): the columns [gout_c0, ncols) are a layer's complete dY --
  // store its dYpre instead and sum the dalpha / dbias partials of the tile
  // (the launcher takes gate-out only with COLFIX, full tiles and 16-B units)
  const bool go = COLFIX && d.gout != nullptr;
  float oalpha[VEC];   // slopes of the gated layer for this thread's channels (COLFIX)
  const int ccol = n0 + (tid % UPR) * VEC;
  {
    const bool g_on = go && ccol >= d.gout_c0 && ccol < d.ncols;
#pragma unroll
    for (int q = 0; q < VEC; ++q) oalpha[q] = g_on ? d.gout_alpha[ccol - d.gout_c0 + q] : 0.f;
  }
  float* const Ct = (float*)lds;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jn = 0; jn < NTL; ++jn)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Ct[((wm * WTM + i * 16 + g * 4 + e) * CROW) / 4 + wn * WTN + jn * 16 + r] = acc[i][jn][e];
  __syncthreads();

  if constexpr (SPLIT) {   // raw fp32 slice of the tile: 16-B units of 4 columns (ncols % 4 == 0)
    float* const wz = ws + (int64_t)blockIdx.y * ((int64_t)d.n * H * W) * d.ncols;
    for (int u = tid; u < BM * (BN / 4); u += NT) {
      const int px = u / (BN / 4), cl = (u - px * (BN / 4)) * 4, c = n0 + cl;
      const int yy = y0 + px / TW, xx = x0 + px % TW;
      if (yy >= H || xx >= W || c >= d.ncols) continue;
      *(f32x4*)(wz + (((int64_t)nimg * H + yy) * W + xx) * d.ncols + c) = *(const f32x4*)(Ct + (px * CROW) / 4 + cl);
    }
    return;
  }
  if (!fast) {
    c3::store_tile<T, BN, NT>(d, Ct, CROW / 4, y0, x0, nimg, n0, tid);
    return;
  }
  float gsa[VEC], gsb[VEC];
#pragma unroll
  for (int q = 0; q < VEC; ++q) { gsa[q] = 0.f; gsb[q] = 0.f; }
  float ebias[VEC], ealpha[VEC];
  int64_t cf_pre = 0, cf_out = 0, cf_res = 0;
  if constexpr (COLFIX) {
    const int c = ccol;
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      ebias[q] = ((flags & RDN_EPI_BIAS) && c + q < d.ncols) ? d.bias[c + q] : 0.f;
      ealpha[q] = ((flags & RDN_EPI_PRELU) && c + q < d.ncols) ? d.alpha[c + q] : 0.f;
    }
    cf_pre = rdn_coff(c, d.pre_ps, d.pre_pl);
    cf_out = rdn_coff(d.out_c0 + c, d.out_ps, d.out_pl);
    cf_res = rdn_coff(d.res_c0 + c, d.res_ps, d.res_pl);
  }
#pragma unroll
  for (int it = 0; it < E_IT; ++it) {
    const int u = tid + it * NT;
    if (it + 1 == E_IT && u >= EU) continue;
    const int px = u / UPR, cl = (u - px * UPR) * VEC, c = n0 + cl;
    if (c >= d.ncols) continue;
    float v[VEC];
    const float* src = Ct + (px * CROW) / 4 + cl;
#pragma unroll
    for (int q = 0; q < VEC; q += 4) {
      const f32x4 t4 = *(const f32x4*)(src + q);
      v[q] = t4[0]; v[q + 1] = t4[1]; v[q + 2] = t4[2]; v[q + 3] = t4[3];
    }
    const int64_t opix = opix0 + (px / TW) * W + px % TW;
    if (flags & RDN_EPI_BIAS) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += COLFIX ? ebias[q] : d.bias[c + q];
    }
    if (flags & RDN_EPI_STORE_PRE)
      *(u32x4*)((T*)d.pre + opix * d.pre_ps + (COLFIX ? cf_pre : rdn_coff(c, d.pre_ps, d.pre_pl))) = Unit16<T>::pack(v);
    if (flags & RDN_EPI_PRELU) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const float a = COLFIX ? ealpha[q] : d.alpha[c + q];
        v[q] = v[q] > 0.f ? v[q] : a * v[q];
      }
    }
    T* const op = (T*)d.out + opix * d.out_ps + (COLFIX ? cf_out : rdn_coff(d.out_c0 + c, d.out_ps, d.out_pl));
    float rv[VEC];
    if ((flags & RDN_EPI_RESID) && c < d.res_climit) {
      Unit16<T>::unpack(*(const u32x4*)((const T*)d.res + opix * d.res_ps +
                                        (COLFIX ? cf_res : rdn_coff(d.res_c0 + c, d.res_ps, d.res_pl))), rv);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += rv[q];
    }
    if (flags & RDN_EPI_ACCUM) {
      Unit16<T>::unpack(*(const u32x4*)op, rv);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += rv[q];
    }
    if (go && c >= d.gout_c0) {   // dYpre = dY * (pre > 0 ? 1 : alpha); aten prelu backward
      const int gc = c - d.gout_c0;
      float pr[VEC];
      Unit16<T>::unpack(*(const u32x4*)((const T*)d.gout_pre + opix * d.gout_pre_ps + gc), pr);
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const bool pos = pr[q] > 0.f;
        if (!pos) gsa[q] += pr[q] * v[q];
        v[q] = pos ? v[q] : oalpha[q] * v[q];
        gsb[q] += v[q];
      }
      *(u32x4*)((T*)d.gout + opix * d.gout_ps + gc) = Unit16<T>::pack(v);
      continue;
    }
    *(u32x4*)op = Unit16<T>::pack(v);
  }
  if (!go || n0 + BN <= d.gout_c0) return;
  // per-channel partials of the tile: the lanes of a wave holding one channel group
  // (lane, lane + UPR, ...) combine by xor shuffles, then the 4 waves through LDS,
  // in a fixed order (the fp32 tile is consumed)
  if constexpr (COLFIX) {
#pragma unroll
    for (int m = UPR; m < 64; m <<= 1)
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        gsa[q] += __shfl_xor(gsa[q], m, 64);
        gsb[q] += __shfl_xor(gsb[q], m, 64);
      }
    __syncthreads();
    float* const red = (float*)lds;   // [wave][2][BN]
    if (lane < UPR) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        red[(wave * 2 + 0) * BN + lane * VEC + q] = gsa[q];
        red[(wave * 2 + 1) * BN + lane * VEC + q] = gsb[q];
      }
    }
    __syncthreads();
    const int gcn = d.ncols - d.gout_c0;
    float* const part = d.gout_part + (int64_t)(lb / ncb) * 2 * gcn;
    for (int j = tid; j < 2 * BN; j += NT) {
      const int which = j / BN, col = j - which * BN, c = n0 + col;
      if (c < d.gout_c0 || c >= d.ncols) continue;
      part[which * gcn + (c - d.gout_c0)] = (red[which * BN + col] + red[(2 + which) * BN + col]) +
                                            (red[(4 + which) * BN + col] + red[(6 + which) * BN + col]);
    }
  }
}

template <typename T, int BN, int WMW, int CK>
int launch_h(const rdn_conv_desc* d, hipStream_t st, int splits = 0, float* ws = nullptr) {
  const int tiles_x = (d->w + TW - 1) / TW, tiles_y = (d->h + TH - 1) / TH;
  const int64_t blocks = (int64_t)d->n * tiles_x * tiles_y * ((d->ncols + BN - 1) / BN);
  dim3 grid((unsigned)blocks);
  if (splits > 0) {   // split-K slices (rdn_conv_fwd_splitk); no gate / gate-out here
    const int nch = d->cin / CK, c_per = (nch + splits - 1) / splits;
    RDN_PROBE("conv3_halo_kernel<%s,%d,%d,%d,split>", rdn_tname<T>(), BN, WMW, CK);
    conv3_halo_kernel<T, BN, WMW, CK, false, false, true><<<dim3((unsigned)blocks, (nch + c_per - 1) / c_per), NT, 0, st>>>(
        *d, tiles_x, tiles_y, c_per, ws);
    return rdn_check_launch("rdn_conv_fwd_splitk(conv3)");
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  }
  const bool pair = blocks <= 2 * (int64_t)cus;
  if (d->gout) {
    // gate-out only on the fast epilogue with a fixed channel group per thread
    constexpr int VEC = TypeInfo<T>::VEC;
    const bool colfix = NT % (BN / VEC) == 0 && BN % VEC == 0;
    const bool full = d->h % TH == 0 && d->w % TW == 0 && d->ncols % VEC == 0 && !(d->flags & RDN_EPI_OUT_NCHW) &&
                      d->out_ps % VEC == 0 && d->out_c0 % VEC == 0 &&
                      (!(d->flags & RDN_EPI_RESID) || (d->res_climit % VEC == 0 && d->res_ps % VEC == 0 &&
                                                       d->res_c0 % VEC == 0));
    if (!colfix || !full) {
      rdn_set_error("rdn_conv_fwd(conv3): gate-out needs full 8x16 tiles and a column tile of whole channel groups");
      return RDN_E_SHAPE;
    }
    rdn_probe_rows = (int)(d->n * tiles_x * tiles_y);
  }
  RDN_PROBE("conv3_halo_kernel<%s,%d,%d,%d%s%s>", rdn_tname<T>(), BN, WMW, CK, d->gate ? ",gate" : "",
            pair && sizeof(T) == 2 && BN <= 96 ? ",pair" : "");
  if (d->gate) {
    if constexpr (NT % (CK / TypeInfo<T>::VEC) == 0) {
      if (pair) conv3_halo_kernel<T, BN, WMW, CK, true, true><<<grid, NT, 0, st>>>(*d, tiles_x, tiles_y);
      else conv3_halo_kernel<T, BN, WMW, CK, true, false><<<grid, NT, 0, st>>>(*d, tiles_x, tiles_y);
    } else {
      rdn_set_error("rdn_conv_fwd(conv3): gated input needs a power-of-two channel chunk");
      return RDN_E_SHAPE;
    }
  } else {
    if (pair) conv3_halo_kernel<T, BN, WMW, CK, false, true><<<grid, NT, 0, st>>>(*d, tiles_x, tiles_y);
    else conv3_halo_kernel<T, BN, WMW, CK, false, false><<<grid, NT, 0, st>>>(*d, tiles_x, tiles_y);
  }
  return rdn_check_launch("rdn_conv_fwd(conv3)");
}

// BN choice: 64 for wide outputs (more blocks on the small deep levels; measured
// best on the L1-L3 shapes) unless 80 tiles them exactly and 64 does not, else the
// candidate minimising padded columns
// ceil(ncols/BN)*BN, ties to the larger BN
static int pick_bn_cols(int ncols) {
  if (ncols > 128) return ncols % 64 && ncols % 80 == 0 ? 80 : 64;   // 160 -> 2 x 80 (measured), else 64
  static const int cands[] = {128, 96, 80, 64, 48, 32, 16};
  int best = 128, waste = 1 << 30;
  for (int b : cands) {
    const int w = (ncols + b - 1) / b * b - ncols;
    if (w < waste) { waste = w; best = b; }
  }
  return best;
}

// minimum grid before BN is halved: a 32x32 level-3 layer has only 128 pixel tiles
// per 16 images, so BN=128 would leave half of the 256 CUs idle (A/B on MI355X,
// whole train step: 128 blocks 1351, 256 blocks 1338, 512 blocks 1369 img/s)
constexpr int MIN_BLOCKS = 512;

static int pick_bn(int ncols, int64_t tiles) {
  int bn = pick_bn_cols(ncols);
  while ((bn == 128 || bn == 64) && ncols % (bn / 2) == 0 &&
         tiles * ((ncols + bn - 1) / bn) < (int64_t)MIN_BLOCKS)
    bn /= 2;
  return bn;
}

template <typename T, int CK>
int launch_bn(const rdn_conv_desc* d, hipStream_t st, int splits = 0, float* ws = nullptr) {
  const int64_t tiles = (int64_t)d->n * ((d->h + c3::TH - 1) / c3::TH) * ((d->w + c3::TW - 1) / c3::TW);
  const int bn = d->bn ? d->bn : pick_bn(d->ncols, tiles);
  switch (bn) {
    case 16: return launch_h<T, 16, 4, CK>(d, st, splits, ws);
    case 32: return launch_h<T, 32, 4, CK>(d, st, splits, ws);
    case 48: return launch_h<T, 48, 4, CK>(d, st, splits, ws);
    case 64: return launch_h<T, 64, 2, CK>(d, st, splits, ws);
    case 80: return launch_h<T, 80, 4, CK>(d, st, splits, ws);
    case 96: return launch_h<T, 96, 4, CK>(d, st, splits, ws);
    case 128: return launch_h<T, 128, 2, CK>(d, st, splits, ws);
  }
  rdn_set_error("rdn_conv_fwd(conv3): unsupported bn=%d", bn);
  return RDN_E_ARG;
}

}  // namespace

int rdn_conv3_chunk_pow2(int cin, int cap) {
  int ck = cap;
  while (ck > 8 && (cin % ck)) ck >>= 1;
  return (cin % ck) ? -1 : ck;
}

// K-side channel chunk of the halo conv: the whole pixel row for the narrow
// 48/80/96-channel inputs of level 0 (bf16: one contiguous 96-192 B read per
// pixel instead of 3-6 passes of 32 B), else the largest power of two <= 64 (bf16)
// / 32 (fp32) dividing cin.
int rdn_conv3_chunk_impl(int cin, int dtype) {
  if (dtype == RDN_BF16 && (cin == 48 || cin == 80 || cin == 96)) return cin;
  return rdn_conv3_chunk_pow2(cin, dtype == RDN_BF16 ? 64 : 32);
}

extern "C" int rdn_conv3_chunk(int32_t cin, int32_t dtype) { return rdn_conv3_chunk_impl(cin, dtype); }

extern "C" int rdn_conv3_packed_k(int32_t cin, int32_t dtype) {
  const int ck = rdn_conv3_chunk_impl(cin, dtype);
  if (ck < 0) return RDN_E_SHAPE;
  const int sk = dtype == RDN_BF16 ? 64 : 32;
  const int kc = (9 * ck + sk - 1) / sk * sk;
  const int kp = (cin / ck) * kc;
  return (kp + 63) / 64 * 64;
}

extern "C" int rdn_conv3_pick_bn(int32_t ncols) { return pick_bn_cols(ncols); }

int rdn_conv3_launch(const rdn_conv_desc* d, hipStream_t st) {
  const int ck = rdn_conv3_chunk_impl(d->cin, d->dtype);
  if (d->gate && (!d->gate_alpha || d->gate_ps % (d->dtype == RDN_BF16 ? 8 : 4) || ((uintptr_t)d->gate & 15))) {
    rdn_set_error("rdn_conv_fwd(conv3): gate needs alpha and 16-byte aligned rows"); return RDN_E_ARG;
  }
  if (ck < 0) { rdn_set_error("rdn_conv_fwd(conv3): cin=%d not a multiple of 8", d->cin); return RDN_E_SHAPE; }
  if (d->kp < rdn_conv3_packed_k(d->cin, d->dtype)) {
    rdn_set_error("rdn_conv_fwd(conv3): kp=%d < packed K %d (pack with ck=%d)", d->kp,
                  rdn_conv3_packed_k(d->cin, d->dtype), ck);
    return RDN_E_SHAPE;
  }
  if (d->dtype == RDN_BF16) {
    const int big = rdn_conv3_big_launch(d, ck, st);   // MFMA-heavy level-1..3 shapes (conv3_big.hip)
    if (big <= 0) return big;
    const int wsd = rdn_conv3_wsd_launch(d, ck, st);   // full-tile level-0/1 shapes (conv3_wsd.hip)
    if (wsd <= 0) return wsd;
    const int ws = rdn_conv3_ws_launch(d, ck, st);
    if (ws <= 0) return ws;
    switch (ck) {
      case 96: return launch_bn<bf16, 96>(d, st);
      case 80: return launch_bn<bf16, 80>(d, st);
      case 48: return launch_bn<bf16, 48>(d, st);
      case 64: return launch_bn<bf16, 64>(d, st);
      case 32: return launch_bn<bf16, 32>(d, st);
      case 16: return launch_bn<bf16, 16>(d, st);
      default: return launch_bn<bf16, 8>(d, st);
    }
  }
  switch (ck) {
    case 32: return launch_bn<float, 32>(d, st);
    case 16: return launch_bn<float, 16>(d, st);
    default: return launch_bn<float, 8>(d, st);
  }
}

// ---- split-K slices of the 3x3 forward (round 6; rdn_conv_fwd_splitk, conv_gemm.hip,
// owns the entry point and the reduce): slices for d on this device -- 0 (no split)
// unless the tile grid covers under half of the CUs and there are >= 2 input-channel
// chunks; then enough slices for ~2 blocks per CU, each of >= 1 chunk (rounded so that
// every slice gets the same number of chunks)
int rdn_conv3_splitk_slices(const rdn_conv_desc* d, int cus) {
  if (d->gather != RDN_G_CONV3 || d->gate || d->gout || (d->flags & RDN_EPI_SCATTER2) || d->ncols % 4) return 0;
  const int ck = rdn_conv3_chunk_impl(d->cin, d->dtype);
  if (ck <= 0) return 0;
  const int nch = d->cin / ck;
  const int64_t tiles = (int64_t)d->n * ((d->h + c3::TH - 1) / c3::TH) * ((d->w + c3::TW - 1) / c3::TW);
  const int bn = d->bn ? d->bn : pick_bn(d->ncols, tiles);
  const int64_t base = tiles * ((d->ncols + bn - 1) / bn);
  if (nch < 2 || 2 * base > cus) return 0;
  int s = (int)((rdn_splitk_target(cus) + base - 1) / base);
  if (s > nch) s = nch;
  const int c_per = (nch + s - 1) / s;
  return (nch + c_per - 1) / c_per;
}

// the slice launch: raw fp32 sums of slice y to ws[y][pixel][ncols]
int rdn_conv3_splitk_launch(const rdn_conv_desc* d, int splits, float* ws, hipStream_t st) {
  const int ck = rdn_conv3_chunk_impl(d->cin, d->dtype);
  if (d->dtype == RDN_BF16) {
    switch (ck) {
      case 96: return launch_bn<bf16, 96>(d, st, splits, ws);
      case 80: return launch_bn<bf16, 80>(d, st, splits, ws);
      case 48: return launch_bn<bf16, 48>(d, st, splits, ws);
      case 64: return launch_bn<bf16, 64>(d, st, splits, ws);
      case 32: return launch_bn<bf16, 32>(d, st, splits, ws);
      case 16: return launch_bn<bf16, 16>(d, st, splits, ws);
      default: return launch_bn<bf16, 8>(d, st, splits, ws);
    }
  }
  switch (ck) {
    case 32: return launch_bn<float, 32>(d, st, splits, ws);
    case 16: return launch_bn<float, 16>(d, st, splits, ws);
    default: return launch_bn<float, 8>(d, st, splits, ws);
  }
}
