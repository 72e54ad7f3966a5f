// Declarations shared by the fused DeepFM kernels (dfm_fused.hip: the
// 128-row bf16 kernel, the fp32 kernels and the launcher; dfm_wide.hip: the
// 256-row bf16 kernel of the ITEM plan).
#pragma once

#include "gemm_mfma.h"

namespace hhfm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

constexpr int kFusedMaxLayers = 4;
constexpr int kFusedMaxF = 16;
constexpr int kFusedMaxK = 512;
constexpr int kLdsBytes = 160 * 1024;   // gfx950 LDS per workgroup
constexpr uint64_t kDfmIdentityPerm = 0xFEDCBA9876543210ull;

struct FusedDfmArgs {
  const int32_t* idx;
  int64_t B;
  int F, k;
  const void* E;
  int64_t M;
  const float* w;
  int L;
  int dims[kFusedMaxLayers];
  int ldb[kFusedMaxLayers];
  const uint16_t* Wt[kFusedMaxLayers];
  const float* bias[kFusedMaxLayers];
  const float* Wp;
  float bp;
  float* out;
  const uint4* packed;   // chunk sequence written by dfm_pack_weights
  // PROJ: fp32 P_f[id] at proj + f·proj_fstride + id·proj_ld (f counted from
  // the first projected field), zero beyond
  // dims[0]; fp32 MLP: natural unit order; bf16 MLP: the accumulator order of
  // dfm_proj_pos (a lane's 16 units of a tile are contiguous)
  const void* proj;
  int64_t proj_fstride;
  int proj_ld;           // row stride: projected fields x 32·TM
  int Fd;                // fields [0, Fd) run layer 0 on MFMA, [Fd, F) come from P
                         // (Fd = F: no projection; 0: all fields projected)
  // bf16 kernel: internal field j is the caller's field (perm >> 4j) & 15
  // (direct fields first); row m's score goes to out[order[m]] when order is
  // set (idx then holds the caller's rows regrouped, dfm_order_rows).  The
  // fp32 kernel takes the identity and no order.
  uint64_t perm;
  const int32_t* order;
  // dfm_fused_f32s: base[m] = (Σ_f w·Wp + FM part) + bp from dfm_fm_base;
  // stage: P rows of narrow-span fields staged in LDS (HHFM_PLAN_UNSTAGED: off)
  const float* fmbase;
  int stage;
  // scratch for the FM part's pair table (dfm_fm_pairs); fm_out: its output
  void* scratch;
  size_t scratch_bytes;
  float* fm_out;
  // host side only (never read by a kernel): the call's HHFM_PLAN_* flags and
  // whether the pair table in scratch is already built for this call (the
  // catalog's query chunks build it once)
  int32_t plan;
  bool* pairs_ready;
  // per caller field f of this call's rows (dfm_order_rows): [2f] =
  // 0x7fffffff − min id, [2f+1] = max id, or null; the pair table is then
  // built only in the 128x128 tiles some field pair f < g reads
  const int32_t* franges;
};

HHFM_DEV uint32_t pack_bf16x2(float lo, float hi) {   // v_cvt_pk_bf16_f32 (RNE)
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// One lane-linear 16-B-per-lane LDS-DMA (global_load_lds_dwordx4, M0 = the
// wave's LDS destination) issued through inline asm.  When the compiler sees
// the DMA builtin it treats it as an LDS access of unknown order and drains
// every ds_read with lgkmcnt(0) at each MFMA step boundary; issued this way
// it keeps counted lgkmcnt waits (1 % on C5 ITEM/CTX, profiles/r02_k3_hidden_knockouts.txt).
// The compiler does not track these loads: every barrier that publishes them
// is preceded by an explicit s_waitcnt vmcnt(0) (dma_wait below).
HHFM_DEV void lds_dma16(const void* gsrc, void* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(gsrc), "s"(m0v)
               : "memory");
}

HHFM_DEV void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

HHFM_DEV void swap_halves(uint32_t& a, uint32_t& b) {
  // lanes 32-63 of a <-> lanes 0-31 of b
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

template <bool B>
struct BoolC {
  static constexpr bool value = B;
};

// the 256-row kernel (dfm_wide.hip) at an instantiated shape; false: not
// instantiated (the caller runs dfm_fused)
bool dfm_wide_launch(const FusedDfmArgs& a, int TM, int32_t plan, hipStream_t st);
// bytes of the packed-weight workspace a.packed points to (dfm_fused.hip)
size_t dfm_fused_pack_bytes(int L, const int32_t* dims, bool mlp_bf16);
// base[m] = (Σ_f w·Wp + FM part) + bp into a.fm_out from the pair table
// C = (E ⊙ Wp)·Eᵀ (dfm_fused.hip; built once per call into a.scratch); false
// (nothing launched) when it does not fit a.scratch, the rows are too few to
// pay for it, or the plan asks for HHFM_PLAN_ROW_FM.  base = false: the table
// only (the wide kernel forms the rows' base itself)
bool dfm_fm_pairs(const FusedDfmArgs& a, bool tbf, hipStream_t st, bool base = true);
// split-bf16 hidden layers for the fp32 MLP (no HHFM_PLAN_EXACT_FP32)
inline bool dfm_f32_split(int32_t plan) { return !(plan & HHFM_PLAN_EXACT_FP32); }

}  // namespace hhfm
