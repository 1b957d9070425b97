#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_i8, int8_t) }
