#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_f16, _Float16) }
