#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE_FP(gLaunch_f16, _Float16) }
