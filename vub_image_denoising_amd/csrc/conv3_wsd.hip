// Level-0/1 3x3 convolution (forward and input gradient) for the narrow, HBM-bound
// layers: weight-stationary, persistent, with the input halos streamed by LDS-DMA
// and the epilogue on its own waves (gfx950).
//
// conv3_ws.hip (the previous form, kept as the fallback for ragged shapes) stages
// each halo global -> VGPR -> LDS with one tile in flight, and the same four waves
// run the MFMAs, the epilogue stores and the loads; at these shapes (100-350 MB per
// launch, little arithmetic) it reached 0.29-0.53 of HBM.  Here a block is 8 waves:
//
//   waves 0-3 (MMA): own the LDS-DMA halo ring.  Per tile they wait for their own
//     DMAs (counted `s_waitcnt vmcnt`), publish with a raw s_barrier, issue the DMA
//     of the tile NS-1 ahead, apply the fused PReLU-backward gate in LDS (GATE: the
//     saved PReLU input arrives by DMA beside dY), run the 9 taps x MFMA against the
//     resident weight panel and write the fp32 tile to the LDS epilogue buffer.
//   waves 4-7 (epilogue): meanwhile finish the PREVIOUS tile from that buffer: bias,
//     PReLU-input store, PReLU, residual / accumulate operand (prefetched one tile
//     ahead into registers), 16-byte NHWC stores.
//
// The MMA waves issue no other vector-memory instruction, so their vmcnt counts
// only DMAs and the ring stays in flight across the barriers; the epilogue waves'
// loads and stores are ordinary compiler-tracked memory operations.  DMAs are inline
// asm (the builtin makes the compiler wait vmcnt(0) before LDS reads of the array).
//
// Halo image: dense rows of CK*2 bytes (a DMA wave-instruction fills 1 KiB
// contiguously); the ds_read_b128 fragment reads (16 consecutive pixels x 64 B) are
// kept (nearly) bank-conflict free by rotating each row's 16-byte units by rot(x),
// x = the pixel's column in the halo row -- applied on the per-lane DMA source
// address (rotations chosen by exhaustive check of the read pattern).
//
// Same packed weights (P[n][tap*CK + ci], KC = roundup(9*CK, 64)) and epilogue
// flags as conv3_ws / conv3_halo; only full 8 x 16 tiles with 16-byte NHWC units
// take this path (the launcher checks).
#include "conv3_tile.h"

#include <stdlib.h>

namespace {

using c3::BM;
using c3::HW_;
using c3::TH;
using c3::TW;

constexpr int NTH = 512;                 // 4 MMA waves + 4 epilogue waves
constexpr int LDS_MAX = 160 * 1024;

__device__ __attribute__((aligned(64))) unsigned int g_wsd_zero[16];

// unit rotation of halo row x (0..17) for a CK-channel image
template <int CK>
__device__ __forceinline__ int rot(int x) {
  constexpr int U = CK / 8;
  if constexpr (CK == 16 || CK == 64) return x % U;
  else if constexpr (CK == 32) return (x >> 1) % U;
  else if constexpr (CK == 96) return ((x >> 2) * 6) % U;
  else return 0;                                       // 8, 48, 80: conflict-free unrotated
}

template <int BN, int CK, bool GATE>
struct WsdCfg {
  static constexpr int U = CK / 8;                     // 16-B units per halo pixel
  static constexpr int RB = CK * 2;
  static constexpr int KC = (9 * CK + 63) / 64 * 64;
  static constexpr int NSTEP = KC / 32;
  static constexpr int WROW = KC * 2 + 32;             // = 32 mod 128: conflict-free B reads
  static constexpr int W_BYTES = BN * WROW;
  static constexpr int HPC = (HW_ * RB + 1023) / 1024; // 1-KiB DMA pieces per halo
  static constexpr int STAGE = (GATE ? 2 : 1) * HPC * 1024;
  static constexpr int CROWF = BN + 4;                 // epilogue fp32 row (floats)
  static constexpr int CT_BYTES = BM * CROWF * 4;
  static constexpr int AL_BYTES = GATE ? (CK * 4 + 15) / 16 * 16 : 0;
  static constexpr int FIXED = W_BYTES + CT_BYTES + AL_BYTES;
  static constexpr int NS = FIXED + 3 * STAGE <= LDS_MAX ? 3 : 2;
  static constexpr int LDS = FIXED + NS * STAGE;
  static constexpr bool FITS = LDS <= LDS_MAX && BN <= 80;   // 96 columns spill (fallback: conv3_ws)
};

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// one LDS-DMA wave-instruction: 16 B per lane from src to LDS byte dst + lane*16
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

// DMAs a wave issues per tile: pieces wave, wave+4, ... < HPC (x2 with the gate)
template <int HPC, int MULT>
__device__ __forceinline__ void wait_own(int wave, bool one_ahead) {
  if (!one_ahead) { wait_vm<0>(); return; }
  switch (wave) {
    case 0: wait_vm<MULT * ((HPC + 3) / 4)>(); break;
    case 1: wait_vm<MULT * ((HPC + 2) / 4)>(); break;
    case 2: wait_vm<MULT * ((HPC + 1) / 4)>(); break;
    default: wait_vm<MULT * (HPC / 4)>(); break;
  }
}

template <int BN, int CK, bool GATE>
__global__ __launch_bounds__(NTH, 1) void conv3_wsd_kernel(rdn_conv_desc d, int tiles_x, int tiles_y, int ntiles) {
  using Cfg = WsdCfg<BN, CK, GATE>;
  constexpr int U = Cfg::U, RB = Cfg::RB, KC = Cfg::KC, WROW = Cfg::WROW, NSTEP = Cfg::NSTEP, NS = Cfg::NS;
  constexpr int HPC = Cfg::HPC, CROWF = Cfg::CROWF;
  constexpr int HPW = (HPC + 3) / 4;                   // max pieces per wave
  constexpr int MT = 2, NTL = BN / 16;                 // 4 MMA waves x 32 tile pixels
  constexpr int VEC = 8;
  constexpr int UPR = BN / VEC, EU = BM * UPR, E_IT = (EU + 255) / 256;
  constexpr bool COLFIX = 256 % UPR == 0;
  static_assert(Cfg::FITS, "LDS");

  __shared__ __attribute__((aligned(1024))) unsigned char lds[Cfg::LDS];
  unsigned char* const ring = lds;                                   // NS x STAGE
  unsigned char* const wl = lds + NS * Cfg::STAGE;                   // resident weights
  float* const Ct = (float*)(wl + Cfg::W_BYTES);                     // epilogue tile
  float* const alds = (float*)(wl + Cfg::W_BYTES + Cfg::CT_BYTES);   // gate slopes

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool mma = wave < 4;
  const int r = lane & 15, g = lane >> 4;
  const int H = d.h, W = d.w, flags = d.flags;

  // this block's tiles: XCD share [t_lo, t_hi) strided by the XCD's block count, so
  // the tiles in flight on one XCD are adjacent and share halo rows through its L2
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7;
  const int t_lo = (int)((int64_t)ntiles * xcd / 8) + (blockIdx.x >> 3);
  const int t_hi = (int)((int64_t)ntiles * (xcd + 1) / 8);
  const int cnt = t_lo < t_hi ? (t_hi - t_lo + per - 1) / per : 0;
  if (cnt == 0) return;
  auto origin = [&](int i, int& oy, int& ox, int& on) {
    int tt = t_lo + i * per;
    const int tx = tt % tiles_x;
    tt /= tiles_x;
    oy = (tt % tiles_y) * TH;
    ox = tx * TW;
    on = tt / tiles_y;
  };

  // ---- resident weights (and gate slopes), plain loads, once
  {
    const bf16* __restrict__ WP = (const bf16*)d.wp;
    constexpr int UPRW = KC / VEC;
    for (int u = tid; u < BN * UPRW; u += NTH) {
      const int n = u / UPRW, k8 = u - n * UPRW;
      *(u32x4*)(wl + n * WROW + k8 * 16) = *(const u32x4*)(WP + (int64_t)n * d.kp + k8 * VEC);
    }
    if constexpr (GATE)
      for (int c = tid; c < CK; c += NTH) alds[c] = d.gate_alpha[c];
  }
  __syncthreads();   // nothing in flight yet

  const bf16* __restrict__ X = (const bf16*)d.x;
  const bf16* __restrict__ Gp = (const bf16*)d.gate;
  const bf16* const zero = (const bf16*)g_wsd_zero;

  // ================= MMA waves: DMA geometry, fragment offsets
  int h_rel[HPW], g_rel[GATE ? HPW : 1], h_y[HPW], h_x[HPW];
  bool h_row[HPW];
  int offA[NSTEP];
  if (mma) {
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int off = (wave + 4 * j) * 1024 + lane * 16;
      const int hr = off / RB, hx = hr % (TW + 2), hy = hr / (TW + 2);
      const int u = ((off % RB) / 16 - rot<CK>(hx) + U) % U;   // logical unit of this physical slot
      h_row[j] = hr < HW_;
      h_y[j] = hy;
      h_x[j] = hx;
      h_rel[j] = (hy * W + hx) * (int)d.x_ps + rdn_coff32(d.x_c0 + u * VEC, (int)d.x_ps, (int)d.x_pl);
      if constexpr (GATE) g_rel[j] = (hy * W + hx) * (int)d.gate_ps + rdn_coff32(u * VEC, (int)d.gate_ps, (int)d.gate_pl);
    }
    // lane (r, g) of k-step j: pixel r of tile rows 2*wave (+1), k = 32 j + 8 g
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      const int k = 32 * j + 8 * g;
      int tap = k / CK;
      const int ci = k - tap * CK;
      tap = tap < 9 ? tap : 8;   // padded k: zero weights, finite operand
      const int ky = tap / 3, kx = tap - 3 * ky;
      const int hx = r + kx;
      offA[j] = ((2 * wave + ky) * (TW + 2) + hx) * RB + (((ci >> 3) + rot<CK>(hx)) % U) * 16;
    }
  }
  auto issue = [&](int i) {   // DMA of tile i into stage i % NS (MMA waves)
    int y0, x0, nimg;
    origin(i, y0, x0, nimg);
    const int64_t hpix0 = ((int64_t)nimg * H + (y0 - 1)) * W + (x0 - 1);
    const bf16* const xb = X + hpix0 * d.x_ps;
    const bf16* const gb = GATE ? Gp + hpix0 * d.gate_ps : nullptr;
    const bool interior = y0 >= 1 && y0 + TH + 1 <= H && x0 >= 1 && x0 + TW + 1 <= W;
    const unsigned st = lds_addr(ring) + (i % NS) * Cfg::STAGE;
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      if (wave + 4 * j >= HPC) break;   // wave-uniform
      const bool ok = h_row[j] & (interior | (((unsigned)(y0 - 1 + h_y[j]) < (unsigned)H) &
                                              ((unsigned)(x0 - 1 + h_x[j]) < (unsigned)W)));
      glds16(ok ? (const void*)(xb + h_rel[j]) : (const void*)zero, st + (wave + 4 * j) * 1024);
      if constexpr (GATE)
        glds16(ok ? (const void*)(gb + g_rel[j]) : (const void*)zero, st + (HPC + wave + 4 * j) * 1024);
    }
  };

  // ================= epilogue waves: output units, per-thread columns
  const int etid = tid - 256;
  int erel[E_IT], ecol[E_IT];
#pragma unroll
  for (int it = 0; it < E_IT; ++it) {
    const int u = (etid < 0 ? 0 : etid) + it * 256;
    const int px = u / UPR;
    erel[it] = (px / TW) * W + px % TW;
    ecol[it] = (u - px * UPR) * VEC;
  }
  const bool has_res = flags & RDN_EPI_RESID, has_acc = flags & RDN_EPI_ACCUM;
  u32x4 eres[E_IT], eacc[E_IT];
  auto prefetch = [&](int i) {
    int y0, x0, nimg;
    origin(i, y0, x0, nimg);
    const int64_t opix0 = ((int64_t)nimg * H + y0) * W + x0;
#pragma unroll
    for (int it = 0; it < E_IT; ++it) {
      const int c = ecol[it];
      if (it + 1 == E_IT && etid + it * 256 >= EU) continue;
      const int64_t opix = opix0 + erel[it];
      if (has_res && c < d.res_climit)
        eres[it] = *(const u32x4*)((const bf16*)d.res + opix * d.res_ps + rdn_coff32(d.res_c0 + c, (int)d.res_ps, (int)d.res_pl));
      if (has_acc && c < d.ncols)
        eacc[it] = *(const u32x4*)((const bf16*)d.out + opix * d.out_ps + rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl));
    }
  };
  float ebias[COLFIX ? VEC : 1], ealpha[COLFIX ? VEC : 1];
  if constexpr (COLFIX) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const int c = ecol[0] + q;
      ebias[q] = ((flags & RDN_EPI_BIAS) && c < d.ncols) ? d.bias[c] : 0.f;
      ealpha[q] = ((flags & RDN_EPI_PRELU) && c < d.ncols) ? d.alpha[c] : 0.f;
    }
  }
  auto epilogue = [&](int i) {
    int y0, x0, nimg;
    origin(i, y0, x0, nimg);
    const int64_t opix0 = ((int64_t)nimg * H + y0) * W + x0;
#pragma unroll
    for (int it = 0; it < E_IT; ++it) {
      const int u = etid + it * 256;
      const int c = ecol[it];
      if ((it + 1 == E_IT && u >= EU) || c >= d.ncols) continue;
      float v[VEC];
      const float* src = Ct + (u / UPR) * CROWF + c;
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
      if (flags & RDN_EPI_STORE_PRE)
        *(u32x4*)((bf16*)d.pre + opix * d.pre_ps + rdn_coff32(c, (int)d.pre_ps, (int)d.pre_pl)) = Unit16<bf16>::pack(v);
      if (flags & RDN_EPI_PRELU) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const float a = COLFIX ? ealpha[q] : d.alpha[c + q];
          v[q] = v[q] > 0.f ? v[q] : a * v[q];
        }
      }
      float rv[VEC];
      if (has_res && c < d.res_climit) {
        Unit16<bf16>::unpack(eres[it], rv);
#pragma unroll
        for (int q = 0; q < VEC; ++q) v[q] += rv[q];
      }
      if (has_acc) {
        Unit16<bf16>::unpack(eacc[it], rv);
#pragma unroll
        for (int q = 0; q < VEC; ++q) v[q] += rv[q];
      }
      *(u32x4*)((bf16*)d.out + opix * d.out_ps + rdn_coff32(d.out_c0 + c, (int)d.out_ps, (int)d.out_pl)) =
          Unit16<bf16>::pack(v);
    }
  };

  // ================= the pipeline (every wave passes the same barriers)
  if (mma) {
    issue(0);
    if (NS == 3 && cnt > 1) issue(1);
  }
  for (int i = 0; i <= cnt; ++i) {
    f32x4 acc[MT][NTL];
    if (mma && i < cnt) wait_own<HPC, GATE ? 2 : 1>(wave, NS == 3 && i + 1 < cnt);   // own DMAs of tile i landed
    wait_lgkm0();                                    // Ct writes of tile i-1 done
    barrier();                                       // A: stage i complete; stage i-1 and Ct(i-1) released
    const unsigned char* const st = ring + (i % NS) * Cfg::STAGE;
    if (mma && i + NS - 1 < cnt) issue(i + NS - 1);
    if constexpr (GATE) {
      if (mma && i < cnt) {   // dY <- dY * (pre > 0 ? 1 : alpha) in place, slot by slot
        unsigned char* const hs = ring + (i % NS) * Cfg::STAGE;
        for (int k = tid; k < HW_ * U; k += 256) {
          const int hr = k / U, ps = k - hr * U;
          const int u = (ps - rot<CK>(hr % (TW + 2)) + U) % U;
          float dy[VEC], pr[VEC];
          Unit16<bf16>::unpack(*(const u32x4*)(hs + k * 16), dy);
          Unit16<bf16>::unpack(*(const u32x4*)(hs + HPC * 1024 + k * 16), pr);
          const f32x4 a0 = *(const f32x4*)(alds + u * VEC), a1 = *(const f32x4*)(alds + u * VEC + 4);
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            const float a = q < 4 ? a0[q] : a1[q - 4];
            dy[q] = pr[q] > 0.f ? dy[q] : a * dy[q];
          }
          *(u32x4*)(hs + k * 16) = Unit16<bf16>::pack(dy);
        }
      }
      wait_lgkm0();
      barrier();                                     // G: gated halo visible
    }
    if (mma && i < cnt) {
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NTL; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      const unsigned char* const pb = wl + r * WROW + g * 16;
      // fragments PF k-steps ahead: one MMA wave per SIMD, so nothing else hides the
      // LDS latency of a step's reads (~100+ cycles) behind its MT x NTL MFMAs
      constexpr int PF = MT * NTL >= 6 ? 1 : MT * NTL >= 4 ? 2 : 4;
      u32x4 fa[NSTEP][MT], fb[NSTEP][NTL];
      auto ld = [&](int j) {
#pragma unroll
        for (int a = 0; a < MT; ++a) fa[j][a] = *(const u32x4*)(st + offA[j] + a * (TW + 2) * RB);
#pragma unroll
        for (int b = 0; b < NTL; ++b) fb[j][b] = *(const u32x4*)(pb + b * 16 * WROW + j * 64);
      };
#pragma unroll
      for (int j = 0; j < PF && j < NSTEP; ++j) ld(j);
#pragma unroll
      for (int j = 0; j < NSTEP; ++j) {
        if (j + PF < NSTEP) ld(j + PF);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < MT; ++a)
#pragma unroll
          for (int b = 0; b < NTL; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[j][a]),
                                                                __builtin_bit_cast(bf16x8, fb[j][b]), acc[a][b], 0, 0, 0);
      }
    }
    if (!mma) {
      if (i >= 1) epilogue(i - 1);
      if (i < cnt && (has_res || has_acc)) prefetch(i);
    }
    wait_lgkm0();
    barrier();                                       // B: Ct(i-1) consumed
    if (mma && i < cnt) {
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NTL; ++b)
#pragma unroll
          for (int e = 0; e < 4; ++e) Ct[(wave * 32 + a * 16 + g * 4 + e) * CROWF + b * 16 + r] = acc[a][b][e];
    }
  }
}

template <typename K>
int resident_per_cu(K kernel) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, NTH, 0) != hipSuccess || n < 1) n = 1;
  return n < 2 ? n : 2;
}

template <int BN, int CK>
int launch_wsd(const rdn_conv_desc* d, hipStream_t st) {
  const bool gate = d->gate != nullptr;
  const int tiles_x = d->w / TW, tiles_y = d->h / TH;
  const int64_t nt = (int64_t)d->n * tiles_x * tiles_y;
  if (nt >= (1ll << 31)) return 1;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  }
  auto run = [&](auto kern, const char* tag) -> int {
    RDN_PROBE("conv3_wsd_kernel<bf16,%d,%d%s>", BN, CK, tag);
    static const int bpc = resident_per_cu(kern);
    const int per_xcd = (int)((nt + 7) / 8);
    int slots = cus * bpc / 8;
    if (slots > per_xcd) slots = per_xcd;
    if (slots < 1) slots = 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)(8 * slots)), dim3(NTH), 0, st, *d, tiles_x, tiles_y, (int)nt);
    return rdn_check_launch("rdn_conv_fwd(conv3 wsd)");
  };
  if (gate) {
    if constexpr (WsdCfg<BN, CK, true>::FITS) return run(conv3_wsd_kernel<BN, CK, true>, ",gate");
    return 1;
  }
  if constexpr (WsdCfg<BN, CK, false>::FITS) return run(conv3_wsd_kernel<BN, CK, false>, "");
  return 1;
}

template <int CK>
int wsd_bn(const rdn_conv_desc* d, hipStream_t st) {
  switch ((d->ncols + 15) / 16) {
    case 1: return launch_wsd<16, CK>(d, st);
    case 2: return launch_wsd<32, CK>(d, st);
    case 3: return launch_wsd<48, CK>(d, st);
    case 4: return launch_wsd<64, CK>(d, st);
    case 5: return launch_wsd<80, CK>(d, st);
    case 6: return launch_wsd<96, CK>(d, st);
  }
  return 1;
}

}  // namespace

// 0 = launched, < 0 = error, 1 = not served here (caller falls back to conv3_ws)
int rdn_conv3_wsd_launch(const rdn_conv_desc* d, int ck, hipStream_t st) {
  static const bool off = [] {
    const char* e = getenv("RDN_CONV3_WSD");
    return e && e[0] == '0';
  }();
  if (off || d->dtype != RDN_BF16 || d->bn || ck != d->cin || d->ncols > 96 || d->ncols % 8 || d->gout) return 1;
  // where it beats conv3_ws (per-layer A/B on the train step, r02): the forward
  // convs with 96-channel inputs (level-1 conv_1 46 -> 32 us, up_0 123 -> 112 us)
  // and the 64 -> 32 level-1 forward; elsewhere conv3_ws's 2-3 resident blocks per
  // CU hide more latency, and the gated input gradients (80 columns: 138 -> 128 us
  // alone) lost it again beside the weight-gradient stream
  const int bn16 = (d->ncols + 15) / 16 * 16;
  if (d->gate || !(ck == 96 || (bn16 == 32 && ck == 64))) return 1;
  if (d->h % TH || d->w % TW) return 1;                          // full tiles only
  const int flags = d->flags;
  if (flags & (RDN_EPI_OUT_NCHW | RDN_EPI_SCATTER2)) return 1;
  if ((flags & RDN_EPI_RESID) && (d->res_climit % 8 || d->res_ps % 8 || d->res_c0 % 8 || ((uintptr_t)d->res & 15)))
    return 1;
  if (d->out_ps % 8 || d->out_c0 % 8 || ((uintptr_t)d->out & 15)) return 1;
  if ((flags & RDN_EPI_STORE_PRE) && (d->pre_ps % 8 || ((uintptr_t)d->pre & 15))) return 1;
  if (d->x_ps % 8 || d->x_c0 % 8 || ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15) || d->kp % 8) return 1;
  if (d->gate && (d->gate_ps % 8 || ((uintptr_t)d->gate & 15))) return 1;
  switch (ck) {
    case 8: return wsd_bn<8>(d, st);
    case 16: return wsd_bn<16>(d, st);
    case 32: return wsd_bn<32>(d, st);
    case 48: return wsd_bn<48>(d, st);
    case 64: return wsd_bn<64>(d, st);
    case 80: return wsd_bn<80>(d, st);
    case 96: return wsd_bn<96>(d, st);
  }
  return 1;
}
