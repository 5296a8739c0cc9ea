// Shared device helpers for librdunet_hip (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/rdunet_hip.h"

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// two floats -> one dword of two bf16 (low, high) by ONE v_cvt_pk_bf16_f32 (RNE).  The
// per-element form (two scalar casts, shift, or) compiles to two cvts with a zero second
// operand plus the merge: 4 VALU per pair instead of 1, same bits
__device__ __forceinline__ unsigned rdn_cvt2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}

#define RDN_LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

template <typename T> struct TypeInfo;
template <> struct TypeInfo<float> { static constexpr int VEC = 4; };
template <> struct TypeInfo<bf16> { static constexpr int VEC = 8; };

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

// 16-byte unit <-> floats
template <typename T> struct Unit16;
template <> struct Unit16<float> {
  static constexpr int N = 4;
  // NOTE: whole-vector bit casts only.  hipcc (ROCm 7.2) miscompiles
  // __builtin_bit_cast(float, v[i]) on an ext_vector element: it returns v[0].
  __device__ static void unpack(const u32x4& u, float* f) {
    const f32x4 v = __builtin_bit_cast(f32x4, u);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = v[i];
  }
  __device__ static u32x4 pack(const float* f) {
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = f[i];
    return __builtin_bit_cast(u32x4, v);
  }
};
__device__ __forceinline__ float bf16lo(unsigned int w) { return __builtin_bit_cast(float, w << 16); }
__device__ __forceinline__ float bf16hi(unsigned int w) { return __builtin_bit_cast(float, w & 0xffff0000u); }
template <> struct Unit16<bf16> {
  static constexpr int N = 8;
  __device__ static void unpack(const u32x4& u, float* f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = bf16lo(u[i]); f[2 * i + 1] = bf16hi(u[i]); }
  }
  __device__ static u32x4 pack(const float* f) {
    u32x4 u;
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = rdn_cvt2(f[2 * i], f[2 * i + 1]);
    return u;
  }
};

// Element offset of channel c (counted across planes) within a pixel of an operand
// with pixel stride ps and plane stride pl (include/rdunet_hip.h: pl == 0 is plain
// NHWC, else channels come in [pixels][ps] planes).  A 16-byte unit never
// straddles two planes (ps % VEC == 0), so offset(c + q) = offset(c) + q inside it.
__host__ __device__ __forceinline__ int64_t rdn_coff(int c, int64_t ps, int64_t pl) {
  return pl ? (int64_t)(c / (int)ps) * pl + (c % (int)ps) : (int64_t)c;
}

// 32-bit form for per-thread offsets the launchers have checked to stay below 2^31
__device__ __forceinline__ int rdn_coff32(int c, int ps, int pl) { return pl ? (c / ps) * pl + (c % ps) : c; }

// XCD-aware block order (MI355X: workgroups are dispatched round-robin over the 8
// XCDs, each with its own L2): logical ids [k*nb/8, (k+1)*nb/8) all run on XCD k,
// so consecutive logical blocks -- which the kernels make share input tiles --
// meet in one L2.  Bijective for any nb (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int xcd = b & 7, q = nb >> 3, r = nb & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// 16-byte load through a buffer descriptor on a wave-uniform base: a byte offset
// past the descriptor's range (OOB) returns zeros -- halo padding without branches,
// so the compiler's vmcnt waits stay exact (a predicated flat load became a branch
// with a vmcnt(0) inside)
constexpr int RDN_OOB = 0x7ffffff0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rdn_rsrc(const void* base) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, RDN_OOB, 0x00020000);
}
// a descriptor of zero records: every access through it is out of range (stores dropped,
// loads 0) -- the PReLU-input stores of a forward-only engine, which keeps none
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rdn_rsrc_none(const void* base) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, 0, 0x00020000);
}
__device__ __forceinline__ u32x4 rdn_ld16(__amdgpu_buffer_rsrc_t rs, bool ok, int off_bytes) {
  int o = ok ? off_bytes : RDN_OOB;
  asm volatile("" : "+v"(o));   // opaque: keeps ONE load (hipcc otherwise splits it into two predicated ones)
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
}

__device__ __forceinline__ u32x2 rdn_ld8(__amdgpu_buffer_rsrc_t rs, bool ok, int off_bytes) {
  int o = ok ? off_bytes : RDN_OOB;
  asm volatile("" : "+v"(o));
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 0));
}
// 4 floats -> 4 bf16 (round to nearest even), as Unit16<bf16>::pack
__device__ __forceinline__ u32x2 rdn_pack4(const float* f) {
  u32x2 u;
#pragma unroll
  for (int i = 0; i < 2; ++i) u[i] = rdn_cvt2(f[2 * i], f[2 * i + 1]);
  return u;
}

// PReLU backward of two bf16 channels packed in a dword (aten _prelu_kernel_backward
// with a bf16 output): dYpre = pre > 0 ? dY : bf16(alpha * dY).  `pre > 0` from the
// bf16 bit pattern b, per 16-bit half: (u16)(b - 1) < 0x7F80 -- +0, -0, negatives
// and NaN take the slope branch, exactly as the fp32 compare does -- as the sign of
// sat_u16((b - 1) + 0x80), spread to a 16-bit mask by an arithmetic shift (inline
// asm: hipcc turns the vector form back into per-half compares and selects).  The
// positive halves keep dY's bits; the others are the RNE-rounded product.
__device__ __forceinline__ unsigned rdn_gate2(unsigned dy, unsigned pre, float alo, float ahi) {
  unsigned m;
  asm("v_pk_sub_u16 %0, %1, %2\n\tv_pk_add_u16 %0, %0, %3 clamp\n\tv_pk_ashrrev_i16 %0, %4, %0"
      : "=&v"(m)
      : "v"(pre), "s"(0x00010001u), "s"(0x00800080u), "s"(0x000f000fu));
  const float lo = __builtin_bit_cast(float, dy << 16) * alo, hi = __builtin_bit_cast(float, dy & 0xffff0000u) * ahi;
  const unsigned g = rdn_cvt2(lo, hi);
  return (g & m) | (dy & ~m);
}

// Fast unsigned division by a runtime-invariant divisor (n < 2^31).
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t t = __umulhi(n, f.m);
  return (t + n) >> f.s;
}

int rdn_conv3_launch(const rdn_conv_desc* d, hipStream_t st);
int rdn_conv3_chunk_impl(int cin, int dtype);
int rdn_conv3_chunk_pow2(int cin, int cap);
int rdn_dense3_l1_launch(const rdn_dense3_desc* d, hipStream_t st);
// blocks a split-K forward launch aims for (conv3_halo.hip / conv_gemm.hip split rules):
// RDN_SPLITK_TARGET blocks per CU (default 1: config 1's graph forward 1.08 -> 1.05 ms
// against 2, r06 -- an fp32 slice block is MFMA-bound, so a launch of more blocks than
// CUs ran its split conv_3 layers in ~16 us instead of ~9.  Slices cut at weight-stage
// instead of chunk granularity measured slower: 1.07 ms at 1, 1.18 at 2)
inline int64_t rdn_splitk_target(int cus) {
  static const int per = [] {
    const char* e = getenv("RDN_SPLITK_TARGET");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 1;
  }();
  return (int64_t)per * cus;
}
int rdn_conv3_splitk_slices(const rdn_conv_desc* d, int cus);
int rdn_conv_pix_launch(const rdn_conv_desc* d, hipStream_t st);
int rdn_conv3_splitk_launch(const rdn_conv_desc* d, int splits, float* ws, hipStream_t st);
int rdn_conv3_ws_launch(const rdn_conv_desc* d, int ck, hipStream_t st);
int rdn_conv3_wsd_launch(const rdn_conv_desc* d, int ck, hipStream_t st);
int rdn_conv3_big_launch(const rdn_conv_desc* d, int ck, hipStream_t st);
int rdn_wgrad3_launch(const rdn_wgrad_desc* d, hipStream_t st);
int rdn_wgrad3_splits(const rdn_wgrad_desc* d);
int rdn_wgrad3_chunks(const rdn_wgrad_desc* d);
int rdn_wgrad3_glds_pick(const rdn_wgrad_desc* d, int single_chunk, int* bm, int* ck);
int rdn_wgrad3_glds_launch(const rdn_wgrad_desc* d, int bm, int ck, int blocks, int tiles_x, int tiles_y, int ntiles,
                           int tpb, hipStream_t st);

// error plumbing (host)
void rdn_set_error(const char* fmt, ...);
int rdn_check_launch(const char* what);

// launch probe (rdn_conv_kernel_name / rdn_wgrad_kernel_name): while set, the
// launchers write the name of the kernel instantiation they would launch and
// return without launching
extern thread_local char* rdn_probe_buf;
extern thread_local int rdn_probe_len;
// rdn_conv_gate_rows: the launcher that would run sets the gate-out partial rows here
extern thread_local int rdn_probe_rows;
int rdn_probe_name(const char* fmt, ...);
#define RDN_PROBE(...) \
  do {                 \
    if (rdn_probe_buf) return rdn_probe_name(__VA_ARGS__); \
  } while (0)
template <typename T> constexpr const char* rdn_tname() { return sizeof(T) == 2 ? "bf16" : "f32"; }
