#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE_FP(gLaunch_f32, float) }
