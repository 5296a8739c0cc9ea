// Pieces shared by the two 3x3 implicit-GEMM kernels (conv3_halo.hip: weights
// streamed per K stage; conv3_ws.hip: weights resident, persistent over tiles):
// the 8 x 16 output-pixel tile geometry, the halo row stride and the epilogue
// that turns an fp32 tile staged in LDS into 16-byte NHWC stores.
#pragma once
#include "rdn_common.h"

namespace c3 {

constexpr int TH = 8, TW = 16, BM = TH * TW;
constexpr int HW_ = (TH + 2) * (TW + 2);   // halo pixels

// halo row stride (bytes) for a CKB-byte pixel row: conflict-free ds_read_b128 for the
// (16 consecutive pixels) x (lane-group 16-B offset) fragment pattern
template <int CKB> struct HaloRow {
  static constexpr int V = CKB <= 32 ? CKB : CKB == 64 ? 96 : CKB == 96 ? 96 : CKB == 128 ? 160
                         : CKB == 160 ? 160 : CKB == 192 ? 224 : CKB + 32;
};

// Epilogue of one 16-byte output unit (VEC channels c.. of pixel opix = (nimg, yy, xx)),
// v = fp32 accumulators.  Applies, per d.flags: bias, pre-activation store, PReLU,
// residual add, accumulate-into-output, NCHW fp32 output.  pf: the residual
// (pf_kind PF_RES) or current-output (PF_ACC) unit already loaded by the caller
// (full NHWC units only); PF_NONE loads it here.
enum { PF_NONE = 0, PF_RES = 1, PF_ACC = 2 };
template <typename T>
__device__ __forceinline__ void finish_unit(const rdn_conv_desc& d, float* v, int c, int64_t opix, int yy, int xx,
                                            int nimg, int pf_kind, u32x4 pf) {
  constexpr int VEC = TypeInfo<T>::VEC;
  const int flags = d.flags;
  const bool full = c + VEC <= d.ncols;
  if (flags & RDN_EPI_BIAS) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] += (c + q < d.ncols) ? d.bias[c + q] : 0.f;
  }
  if (flags & RDN_EPI_STORE_PRE) {
    T* pp = (T*)d.pre + opix * d.pre_ps + rdn_coff(c, d.pre_ps, d.pre_pl);
    if (full) *(u32x4*)pp = Unit16<T>::pack(v);
    else {
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        if (c + q < d.ncols) pp[q] = from_f32<T>(v[q]);
    }
  }
  if (flags & RDN_EPI_PRELU) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const float a = (c + q < d.ncols) ? d.alpha[c + q] : 0.f;
      v[q] = v[q] > 0.f ? v[q] : a * v[q];
    }
  }
  if (flags & RDN_EPI_OUT_NCHW) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      if (c + q >= d.ncols) continue;
      const int64_t o = (((int64_t)nimg * d.cout + c + q) * d.h + yy) * d.w + xx;
      float w = v[q];
      if (flags & RDN_EPI_RESID) w += d.res_nchw[o];
      if (flags & RDN_EPI_ACCUM) w += d.out_nchw[o];
      d.out_nchw[o] = w;
    }
    return;
  }
  if (flags & RDN_EPI_RESID) {
    const T* rp = (const T*)d.res + opix * d.res_ps + rdn_coff(d.res_c0 + c, d.res_ps, d.res_pl);
    if (full && c + VEC <= d.res_climit) {
      float rv[VEC];
      Unit16<T>::unpack(pf_kind == PF_RES ? pf : *(const u32x4*)rp, rv);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += rv[q];
    } else {
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        if (c + q < d.res_climit && c + q < d.ncols) v[q] += to_f32(rp[q]);
    }
  }
  T* op = (T*)d.out + opix * d.out_ps + rdn_coff(d.out_c0 + c, d.out_ps, d.out_pl);
  if (full) {
    if (flags & RDN_EPI_ACCUM) {
      float ov[VEC];
      Unit16<T>::unpack(pf_kind == PF_ACC ? pf : *(const u32x4*)op, ov);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[q] += ov[q];
    }
    *(u32x4*)op = Unit16<T>::pack(v);
  } else {
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      if (c + q >= d.ncols) continue;
      float w = v[q];
      if (flags & RDN_EPI_ACCUM) w += to_f32(op[q]);
      op[q] = from_f32<T>(w);
    }
  }
}

// Epilogue of one BM x PCOLS column slice [c_base, c_base + PCOLS) of an output
// tile.  Ct holds the fp32 accumulators, row p (tile pixel) at Ct[p * crow_f + c],
// c relative to c_base.
template <typename T, int PCOLS, int NT>
__device__ __forceinline__ void store_tile(const rdn_conv_desc& d, const float* Ct, int crow_f, int y0, int x0,
                                           int nimg, int c_base, int tid) {
  constexpr int VEC = TypeInfo<T>::VEC;
  if (d.flags & RDN_EPI_OUT_NCHW) {
    // the network's last conv (fp32 NCHW output + input residual, a few channels): one
    // (channel, pixel) per thread, pixel fastest, so a wave's output / residual accesses
    // are runs of consecutive x in one plane (round 6; through finish_unit a thread took
    // a 16-byte unit of VEC channels of one pixel, nearly all of them padding, and wrote
    // its 3 valid channels to 3 planes: 1.5 TB/s)
    const int nc = d.ncols - c_base < PCOLS ? d.ncols - c_base : PCOLS;
    const int flags = d.flags;
#pragma nounroll
    for (int u = tid; u < nc * BM; u += NT) {
      const int cl = u / BM, p = u - cl * BM;
      const int yy = y0 + p / TW, xx = x0 + p % TW;
      if (yy >= d.h || xx >= d.w) continue;
      const int c = c_base + cl;
      float v = Ct[p * crow_f + cl];
      if (flags & RDN_EPI_BIAS) v += d.bias[c];
      const int64_t opix = ((int64_t)nimg * d.h + yy) * d.w + xx;
      if (flags & RDN_EPI_STORE_PRE) ((T*)d.pre)[opix * d.pre_ps + rdn_coff(c, d.pre_ps, d.pre_pl)] = from_f32<T>(v);
      if (flags & RDN_EPI_PRELU) v = v > 0.f ? v : d.alpha[c] * v;
      const int64_t o = (((int64_t)nimg * d.cout + c) * d.h + yy) * d.w + xx;
      if (flags & RDN_EPI_RESID) v += d.res_nchw[o];
      if (flags & RDN_EPI_ACCUM) v += d.out_nchw[o];
      d.out_nchw[o] = v;
    }
    return;
  }
  constexpr int UPR = PCOLS / VEC;   // 16-B units per tile row
  constexpr int E_UNITS = BM * UPR;
#pragma nounroll
  for (int u = tid; u < E_UNITS; u += NT) {
    const int p = u / UPR, cu = u - p * UPR;
    const int yy = y0 + p / TW, xx = x0 + p % TW;
    const int c = c_base + cu * VEC;
    if (yy >= d.h || xx >= d.w || c >= d.ncols) continue;
    const int64_t opix = ((int64_t)nimg * d.h + yy) * d.w + xx;
    float v[VEC];
    const float* src = Ct + p * crow_f + cu * VEC;
#pragma unroll
    for (int q = 0; q < VEC; q += 4) {
      const f32x4 t4 = *(const f32x4*)(src + q);
      v[q] = t4[0]; v[q + 1] = t4[1]; v[q + 2] = t4[2]; v[q + 3] = t4[3];
    }
    finish_unit<T>(d, v, c, opix, yy, xx, nimg, PF_NONE, u32x4{0u, 0u, 0u, 0u});
  }
}

}  // namespace c3
