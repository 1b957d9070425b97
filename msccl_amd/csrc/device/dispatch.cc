// ncclDataType_t x device reduction op x protocol -> kernel launcher
#include "devcomm.h"

namespace msccl {
#define MSCCL_DECL(N) extern LaunchFn N[6][3]; extern LaunchFn N##_small[2][4]; extern LaunchFn N##_fold[4]; \
  extern LaunchFn N##_pair[4]; extern LaunchFn N##_two[4]; extern LaunchFn N##_direct[4]; extern OneRankFn N##_one; \
  extern const uint32_t N##_layout;
MSCCL_DECL(gLaunch_i8)
MSCCL_DECL(gLaunch_u8)
MSCCL_DECL(gLaunch_i32)
MSCCL_DECL(gLaunch_u32)
MSCCL_DECL(gLaunch_i64)
MSCCL_DECL(gLaunch_u64)
MSCCL_DECL(gLaunch_f16)
MSCCL_DECL(gLaunch_f32)
MSCCL_DECL(gLaunch_f64)
MSCCL_DECL(gLaunch_bf16)

// devOp: 0..3 Sum/Prod/Max/Min, 4 PreMulSum, 5 SumPostDiv (ncclDevRedOp_t, devcomm.h)
LaunchFn getLaunchFn(int dtype, int devOp, int proto) {
  if (devOp < 0 || devOp > 5 || proto < 0 || proto > 2) return nullptr;
  LaunchFn(*tabs[10])[3] = {gLaunch_i8, gLaunch_u8, gLaunch_i32, gLaunch_u32, gLaunch_i64,
                            gLaunch_u64, gLaunch_f16, gLaunch_f32, gLaunch_f64, gLaunch_bf16};
  if (dtype < 0 || dtype > 9) return nullptr;
  return tabs[dtype][devOp][proto];
}

// the small-call kernel (mscclSmallKernel): LL, devOp Sum..Min, transfer set kSetAll / kSetExchange
LaunchFn getSmallLaunchFn(int dtype, int devOp, int set) {
  LaunchFn(*tabs[10])[4] = {gLaunch_i8_small, gLaunch_u8_small, gLaunch_i32_small, gLaunch_u32_small,
                            gLaunch_i64_small, gLaunch_u64_small, gLaunch_f16_small, gLaunch_f32_small,
                            gLaunch_f64_small, gLaunch_bf16_small};
  if (dtype < 0 || dtype > 9 || devOp < 0 || devOp > 3 || set < 0 || set > 1) return nullptr;
  return tabs[dtype][set][devOp];
}

// the flat tree's fold kernel (mscclFoldKernel): LL, devOp Sum..Min
LaunchFn getFoldLaunchFn(int dtype, int devOp) {
  LaunchFn* tabs[10] = {gLaunch_i8_fold, gLaunch_u8_fold, gLaunch_i32_fold, gLaunch_u32_fold, gLaunch_i64_fold,
                        gLaunch_u64_fold, gLaunch_f16_fold, gLaunch_f32_fold, gLaunch_f64_fold, gLaunch_bf16_fold};
  if (dtype < 0 || dtype > 9 || devOp < 0 || devOp > 3) return nullptr;
  return tabs[dtype][devOp];
}

// the pair kernel (mscclPairKernel): LL, devOp Sum..Min
LaunchFn getPairLaunchFn(int dtype, int devOp) {
  LaunchFn* tabs[10] = {gLaunch_i8_pair, gLaunch_u8_pair, gLaunch_i32_pair, gLaunch_u32_pair, gLaunch_i64_pair,
                        gLaunch_u64_pair, gLaunch_f16_pair, gLaunch_f32_pair, gLaunch_f64_pair, gLaunch_bf16_pair};
  if (dtype < 0 || dtype > 9 || devOp < 0 || devOp > 3) return nullptr;
  return tabs[dtype][devOp];
}

// the two-phase fold (mscclTwoPhaseKernel): LL, devOp Sum..Min
LaunchFn getTwoPhaseLaunchFn(int dtype, int devOp) {
  LaunchFn* tabs[10] = {gLaunch_i8_two, gLaunch_u8_two, gLaunch_i32_two, gLaunch_u32_two, gLaunch_i64_two,
                        gLaunch_u64_two, gLaunch_f16_two, gLaunch_f32_two, gLaunch_f64_two, gLaunch_bf16_two};
  if (dtype < 0 || dtype > 9 || devOp < 0 || devOp > 3) return nullptr;
  return tabs[dtype][devOp];
}

// the direct form (mscclDirectKernel): Simple schedules, devOp Sum..Min
LaunchFn getDirectLaunchFn(int dtype, int devOp) {
  LaunchFn* tabs[10] = {gLaunch_i8_direct, gLaunch_u8_direct, gLaunch_i32_direct, gLaunch_u32_direct,
                        gLaunch_i64_direct, gLaunch_u64_direct, gLaunch_f16_direct, gLaunch_f32_direct,
                        gLaunch_f64_direct, gLaunch_bf16_direct};
  if (dtype < 0 || dtype > 9 || devOp < 0 || devOp > 3) return nullptr;
  return tabs[dtype][devOp];
}

const char* kernelLayoutMismatch() {
  const uint32_t stamps[10] = {gLaunch_i8_layout, gLaunch_u8_layout, gLaunch_i32_layout, gLaunch_u32_layout,
                               gLaunch_i64_layout, gLaunch_u64_layout, gLaunch_f16_layout, gLaunch_f32_layout,
                               gLaunch_f64_layout, gLaunch_bf16_layout};
  const char* names[10] = {"int8", "uint8", "int32", "uint32", "int64", "uint64", "float16", "float32", "float64",
                           "bfloat16"};
  for (int i = 0; i < 10; i++)
    if (stamps[i] != kWorkLayout) return names[i];
  return nullptr;
}

OneRankFn getOneRankFn(int dtype) {
  OneRankFn tabs[10] = {gLaunch_i8_one, gLaunch_u8_one, gLaunch_i32_one, gLaunch_u32_one, gLaunch_i64_one,
                        gLaunch_u64_one, gLaunch_f16_one, gLaunch_f32_one, gLaunch_f64_one, gLaunch_bf16_one};
  return dtype >= 0 && dtype <= 9 ? tabs[dtype] : nullptr;
}
}  // namespace msccl
