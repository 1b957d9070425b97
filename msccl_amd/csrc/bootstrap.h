// TCP rendezvous for ncclCommInitRank (replaces the reference's bootstrap.cc:22-462 for one node).
//
// ncclGetUniqueId starts a root thread listening on a TCP port; the 128-byte id carries
// {magic, IPv4 address, port, nonce}.  Every rank connects once and keeps the socket for the
// communicator's lifetime; collective exchanges are rounds in which every rank sends one
// message and the root answers with the concatenation (allgather), which also serves as a
// barrier.  The root thread exits when all ranks have said goodbye.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/nccl.h"

namespace msccl {

struct BootstrapId {
  uint64_t magic;
  uint32_t addr;   // network byte order
  uint16_t port;   // network byte order
  uint16_t pad;
  uint64_t nonce;
};
constexpr uint64_t kBootMagic = 0x424f4f544d534343ull;

ncclResult_t bootstrapCreateRoot(ncclUniqueId* id);

class Bootstrap {
 public:
  virtual ~Bootstrap() {}
  virtual ncclResult_t allgather(const void* mine, size_t bytes, std::vector<char>* all) = 0;
  ncclResult_t barrier() {
    std::vector<char> all;
    char z = 0;
    return allgather(&z, 1, &all);
  }
  int rank = 0, nRanks = 1;
};

class SocketBootstrap : public Bootstrap {
 public:
  ~SocketBootstrap() override;
  static ncclResult_t connect(const ncclUniqueId& id, int rank, int nRanks, SocketBootstrap** out);
  ncclResult_t allgather(const void* mine, size_t bytes, std::vector<char>* all) override;

 private:
  int fd = -1;
};

// Test hook: allgather of one int per rank through a fresh root, no GPU involved.
}  // namespace msccl
