// ncclDataType_t x ncclRedOp_t x protocol -> kernel launcher
#include "devcomm.h"

namespace msccl {
extern LaunchFn gLaunch_i8[4][3], gLaunch_u8[4][3], gLaunch_i32[4][3], gLaunch_u32[4][3], gLaunch_i64[4][3],
    gLaunch_u64[4][3], gLaunch_f16[4][3], gLaunch_f32[4][3], gLaunch_f64[4][3], gLaunch_bf16[4][3];

LaunchFn getLaunchFn(int dtype, int redop, int proto) {
  if (redop < 0 || redop > 3 || proto < 0 || proto > 2) return nullptr;
  LaunchFn(*tabs[10])[3] = {gLaunch_i8, gLaunch_u8, gLaunch_i32, gLaunch_u32, gLaunch_i64,
                            gLaunch_u64, gLaunch_f16, gLaunch_f32, gLaunch_f64, gLaunch_bf16};
  if (dtype < 0 || dtype > 9) return nullptr;
  return tabs[dtype][redop][proto];
}
}  // namespace msccl
