#include "debug.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <pwd.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>

namespace msccl {

namespace {
std::once_flag gOnce;
int gLevel = kLogNone;
uint64_t gMask = kSubInit | kSubEnv;  // reference default mask (debug.cc: INIT,ENV)
FILE* gFile = nullptr;
std::mutex gMu;
thread_local char gLast[1024] = "";
char gHost[64] = "";

std::once_flag gEnvOnce;

void initLog() {
  initEnv();
  const char* lvl = getenv("NCCL_DEBUG");
  if (lvl) {
    if (!strcasecmp(lvl, "VERSION")) gLevel = kLogVersion;
    else if (!strcasecmp(lvl, "WARN")) gLevel = kLogWarn;
    else if (!strcasecmp(lvl, "INFO")) gLevel = kLogInfo;
    else if (!strcasecmp(lvl, "ABORT")) gLevel = kLogAbort;
    else if (!strcasecmp(lvl, "TRACE")) gLevel = kLogTrace;
  }
  const char* sub = getenv("NCCL_DEBUG_SUBSYS");
  if (sub) {
    char* s = strdup(sub);
    bool invert = false;
    if (s[0] == '^') invert = true;
    uint64_t mask = invert ? kSubAll : 0;
    for (char* tok = strtok(s + (invert ? 1 : 0), ","); tok; tok = strtok(nullptr, ",")) {
      struct { const char* n; uint64_t m; } tab[] = {
          {"INIT", kSubInit}, {"COLL", kSubColl}, {"P2P", kSubP2P}, {"SHM", kSubShm},
          {"NET", kSubNet}, {"GRAPH", kSubGraph}, {"TUNING", kSubTune}, {"ENV", kSubEnv},
          {"ALLOC", kSubAlloc}, {"CALL", kSubCall}, {"ALL", kSubAll}};
      for (auto& t : tab)
        if (!strcasecmp(tok, t.n)) mask = invert ? (mask & ~t.m) : (mask | t.m);
    }
    gMask = mask;
    free(s);
  }
  gethostname(gHost, sizeof(gHost) - 1);
  gFile = stdout;
  const char* fn = getenv("NCCL_DEBUG_FILE");
  if (fn && gLevel > kLogVersion) {
    char path[512];
    int o = 0;
    for (int i = 0; fn[i] && o < (int)sizeof(path) - 32; i++) {
      if (fn[i] == '%' && fn[i + 1] == 'h') { o += snprintf(path + o, sizeof(path) - o, "%s", gHost); i++; }
      else if (fn[i] == '%' && fn[i + 1] == 'p') { o += snprintf(path + o, sizeof(path) - o, "%d", getpid()); i++; }
      else path[o++] = fn[i];
    }
    path[o] = 0;
    FILE* f = fopen(path, "w");
    if (f) gFile = f;
  }
}
}  // namespace

const char* lastError() { return gLast; }

// The reference's setEnvFile (misc/param.cc:25-49): one NAME=VALUE per line, split at the first
// '=', a line without '=' skipped, names and values cut at 1023 characters, and an existing
// environment variable never overwritten (setenv(..., 0)).
bool setEnvFile(const char* fileName) {
  FILE* f = fopen(fileName, "r");
  if (f == nullptr) return false;
  char* line = nullptr;
  size_t cap = 0;
  ssize_t len;
  while ((len = getline(&line, &cap, f)) != -1) {
    if (len > 0 && line[len - 1] == '\n') line[--len] = '\0';
    const char* eq = strchr(line, '=');
    if (eq == nullptr) continue;
    std::string name(line, std::min<size_t>(eq - line, 1023));
    std::string value(eq + 1, std::min<size_t>(strlen(eq + 1), 1023));
    setenv(name.c_str(), value.c_str(), 0);
  }
  free(line);
  fclose(f);
  return true;
}

// initEnv (misc/param.cc:51-60), once per process before the first parameter is read:
// ~/.nccl.conf (the passwd entry's home, not $HOME), then /etc/nccl.conf.  The environment wins
// over both, the user's file over the system one.
void initEnv() {
  std::call_once(gEnvOnce, [] {
    const struct passwd* pw = getpwuid(getuid());
    if (pw != nullptr && pw->pw_dir != nullptr) setEnvFile((std::string(pw->pw_dir) + "/.nccl.conf").c_str());
    setEnvFile("/etc/nccl.conf");
  });
}

int64_t envInt(const char* name, int64_t def) {
  initEnv();
  const char* v = getenv(name);
  if (!v || !*v) return def;
  char* end = nullptr;
  long long x = strtoll(v, &end, 0);
  if (end == v) return def;
  return (int64_t)x;
}

void logMessage(int level, uint64_t subsys, const char* file, int line, const char* fmt, ...) {
  std::call_once(gOnce, initLog);
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (level == kLogWarn) snprintf(gLast, sizeof(gLast), "%s", buf);
  if (level > gLevel) return;
  if (level == kLogInfo && !(subsys & gMask)) return;
  if (level == kLogTrace && !(subsys & gMask)) return;
  std::lock_guard<std::mutex> g(gMu);
  int pid = getpid();
  long tid = syscall(SYS_gettid);
  if (level == kLogWarn)
    fprintf(gFile, "\n%s:%d:%ld [msccl-amd] %s:%d NCCL WARN %s\n", gHost, pid, tid, file, line, buf);
  else
    fprintf(gFile, "%s:%d:%ld [msccl-amd] NCCL INFO %s\n", gHost, pid, tid, buf);
  fflush(gFile);
}

}  // namespace msccl
