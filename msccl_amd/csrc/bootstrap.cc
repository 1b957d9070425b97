#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <random>
#include <thread>

#include "debug.h"

namespace msccl {

namespace {

constexpr uint32_t kMsgGoodbye = 0xFFFFFFFFu;

int sendAll(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    c += k;
    n -= k;
  }
  return 0;
}
int recvAll(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    c += k;
    n -= k;
  }
  return 0;
}

struct Hello {
  uint64_t magic, nonce;
  int32_t rank, nRanks;
};

// Root: accept nRanks connections, then serve allgather rounds until every rank said goodbye.
void rootLoop(int lfd, uint64_t nonce) {
  std::vector<int> fds;
  int nRanks = -1;
  std::vector<int> byRank;
  // accept phase (bounded by MSCCL_AMD_BOOTSTRAP_TIMEOUT seconds, default 600)
  int64_t tmo = envInt("MSCCL_AMD_BOOTSTRAP_TIMEOUT", 600);
  time_t start = time(nullptr);
  while (nRanks < 0 || (int)fds.size() < nRanks) {
    struct pollfd pfd = {lfd, POLLIN, 0};
    int r = poll(&pfd, 1, 1000);
    if (time(nullptr) - start > tmo) { WARN("bootstrap root: timed out waiting for ranks"); break; }
    if (r <= 0) continue;
    int fd = accept(lfd, nullptr, nullptr);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    // a connection that never sends its Hello (a stray client, a rank that died while
    // connecting) must not stall the accept loop: bound the read, then drop the socket
    struct timeval tv = {5, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    Hello h;
    if (recvAll(fd, &h, sizeof(h)) || h.magic != kBootMagic || h.nonce != nonce) { close(fd); continue; }
    struct timeval none = {0, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));  // rounds may wait on slow ranks
    if (nRanks < 0) { nRanks = h.nRanks; byRank.assign(nRanks, -1); }
    if (h.nRanks != nRanks || h.rank < 0 || h.rank >= nRanks || byRank[h.rank] != -1) { close(fd); continue; }
    byRank[h.rank] = fd;
    fds.push_back(fd);
  }
  close(lfd);
  if (nRanks < 0 || (int)fds.size() < nRanks) {
    for (int fd : fds) close(fd);
    return;
  }
  // rounds
  std::vector<bool> alive(nRanks, true);
  int nAlive = nRanks;
  while (nAlive > 0) {
    std::vector<std::vector<char>> msgs(nRanks);
    uint32_t len0 = 0;
    bool ok = true;
    int goodbyes = 0;
    for (int r = 0; r < nRanks; r++) {
      if (!alive[r]) continue;
      uint32_t len;
      if (recvAll(byRank[r], &len, 4)) { ok = false; alive[r] = false; nAlive--; continue; }
      if (len == kMsgGoodbye) { alive[r] = false; nAlive--; goodbyes++; close(byRank[r]); continue; }
      msgs[r].resize(len);
      if (len && recvAll(byRank[r], msgs[r].data(), len)) { ok = false; alive[r] = false; nAlive--; continue; }
      len0 = len;
    }
    if (nAlive == 0) break;
    if (goodbyes > 0 || !ok) {
      // a rank left in the middle of a round: nothing consistent to answer; drop everybody
      for (int r = 0; r < nRanks; r++)
        if (alive[r]) close(byRank[r]);
      break;
    }
    std::vector<char> all((size_t)len0 * nRanks);
    for (int r = 0; r < nRanks; r++) {
      if (msgs[r].size() != len0) { ok = false; break; }
      memcpy(all.data() + (size_t)r * len0, msgs[r].data(), len0);
    }
    for (int r = 0; r < nRanks; r++) {
      if (!alive[r]) continue;
      uint32_t len = ok ? (uint32_t)all.size() : 0xFFFFFFFEu;
      if (sendAll(byRank[r], &len, 4) || (ok && sendAll(byRank[r], all.data(), all.size()))) {
        alive[r] = false;
        nAlive--;
      }
    }
  }
}

}  // namespace

ncclResult_t bootstrapCreateRoot(ncclUniqueId* id) {
  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) { WARN("bootstrap: socket() failed: %s", strerror(errno)); return ncclSystemError; }
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  struct sockaddr_in sa;
  memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  const char* host = getenv("MSCCL_AMD_BOOTSTRAP_HOST");
  sa.sin_addr.s_addr = host ? inet_addr(host) : htonl(INADDR_LOOPBACK);
  sa.sin_port = 0;
  if (bind(lfd, (struct sockaddr*)&sa, sizeof(sa)) || listen(lfd, 1024)) {
    WARN("bootstrap: bind/listen failed: %s", strerror(errno));
    close(lfd);
    return ncclSystemError;
  }
  socklen_t sl = sizeof(sa);
  getsockname(lfd, (struct sockaddr*)&sa, &sl);
  BootstrapId bid;
  memset(&bid, 0, sizeof(bid));
  bid.magic = kBootMagic;
  bid.addr = sa.sin_addr.s_addr;
  bid.port = sa.sin_port;
  std::random_device rd;
  bid.nonce = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid();
  memset(id, 0, sizeof(*id));
  memcpy(id->internal, &bid, sizeof(bid));
  std::thread(rootLoop, lfd, bid.nonce).detach();
  INFO(kSubInit, "bootstrap root listening on port %d", ntohs(bid.port));
  return ncclSuccess;
}

ncclResult_t SocketBootstrap::connect(const ncclUniqueId& id, int rank, int nRanks, SocketBootstrap** out) {
  BootstrapId bid;
  memcpy(&bid, id.internal, sizeof(bid));
  if (bid.magic != kBootMagic) { WARN("ncclCommInitRank: invalid unique id"); return ncclInvalidArgument; }
  struct sockaddr_in sa;
  memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = bid.addr;
  sa.sin_port = bid.port;
  int64_t tmo = envInt("MSCCL_AMD_BOOTSTRAP_TIMEOUT", 600);
  time_t start = time(nullptr);
  int fd = -1;
  while (true) {
    fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return ncclSystemError;
    if (::connect(fd, (struct sockaddr*)&sa, sizeof(sa)) == 0) break;
    close(fd);
    fd = -1;
    if (time(nullptr) - start > tmo) { WARN("bootstrap: cannot reach root"); return ncclSystemError; }
    usleep(10000);
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  Hello h = {kBootMagic, bid.nonce, rank, nRanks};
  if (sendAll(fd, &h, sizeof(h))) { close(fd); return ncclSystemError; }
  SocketBootstrap* b = new SocketBootstrap();
  b->fd = fd;
  b->rank = rank;
  b->nRanks = nRanks;
  *out = b;
  return ncclSuccess;
}

ncclResult_t SocketBootstrap::allgather(const void* mine, size_t bytes, std::vector<char>* all) {
  uint32_t len = (uint32_t)bytes;
  if (sendAll(fd, &len, 4) || sendAll(fd, mine, bytes)) { WARN("bootstrap: send failed"); return ncclSystemError; }
  uint32_t rlen;
  if (recvAll(fd, &rlen, 4)) { WARN("bootstrap: root closed the connection"); return ncclSystemError; }
  if (rlen == 0xFFFFFFFEu) { WARN("bootstrap: ranks sent different message sizes"); return ncclInternalError; }
  all->resize(rlen);
  if (rlen && recvAll(fd, all->data(), rlen)) return ncclSystemError;
  return ncclSuccess;
}

SocketBootstrap::~SocketBootstrap() {
  if (fd >= 0) {
    uint32_t bye = kMsgGoodbye;
    sendAll(fd, &bye, 4);
    close(fd);
  }
}

}  // namespace msccl
