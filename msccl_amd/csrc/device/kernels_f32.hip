#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_f32, float) }
