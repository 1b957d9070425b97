// Logging with the reference's env contract: NCCL_DEBUG={VERSION,WARN,INFO,ABORT,TRACE},
// NCCL_DEBUG_SUBSYS (comma list, '^' negates), NCCL_DEBUG_FILE (%h host, %p pid).
// Restates the behaviour of the reference's src/debug.cc:12-185 (not its code).
#pragma once
#include <stdint.h>
#include <string>

namespace msccl {

enum LogLevel { kLogNone = 0, kLogVersion = 1, kLogWarn = 2, kLogInfo = 3, kLogAbort = 4, kLogTrace = 5 };
enum LogSubsys : uint64_t {
  kSubInit = 0x1, kSubColl = 0x2, kSubP2P = 0x4, kSubShm = 0x8, kSubNet = 0x10, kSubGraph = 0x20,
  kSubTune = 0x40, kSubEnv = 0x80, kSubAlloc = 0x100, kSubCall = 0x200, kSubAll = ~0ull
};

void logMessage(int level, uint64_t subsys, const char* file, int line, const char* fmt, ...)
    __attribute__((format(printf, 5, 6)));
// Last WARN text (ncclGetLastError, init.cc:1252-1255)
const char* lastError();
// ~/.nccl.conf and /etc/nccl.conf into the environment, once (misc/param.cc:51-60); every
// parameter read below runs it first.
void initEnv();
// One NAME=VALUE file into the environment without overwriting (misc/param.cc:25-49).
bool setEnvFile(const char* fileName);
// Integer environment parameter (NCCL_PARAM style, param.h:99-108), base prefix accepted.
int64_t envInt(const char* name, int64_t def);

}  // namespace msccl

#define WARN(...) ::msccl::logMessage(::msccl::kLogWarn, ::msccl::kSubAll, __FILE__, __LINE__, __VA_ARGS__)
#define INFO(SUB, ...) ::msccl::logMessage(::msccl::kLogInfo, (SUB), __FILE__, __LINE__, __VA_ARGS__)
#define TRACE(SUB, ...) ::msccl::logMessage(::msccl::kLogTrace, (SUB), __FILE__, __LINE__, __VA_ARGS__)

#define NCCLCHECK(call) do { int _r = (call); if (_r != 0) return (ncclResult_t)_r; } while (0)
#define MSCCLCHECK(call) do { int _r = (call); if (_r != 0) return _r; } while (0)
#define HIPCHECK(call) do { hipError_t _e = (call); if (_e != hipSuccess) { \
    WARN("HIP failure '%s' at %s", hipGetErrorString(_e), #call); return 1; } } while (0)
