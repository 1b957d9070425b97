// Lowering of one-hop MSCCL AllReduce schedules to the flat fold (interpreter.h: runFold).
//
// An msccl-tools schedule is a dataflow program: every rank's thread blocks move chunks through
// per-(channel, peer) FIFOs and fold them with the reduction op (the reference interprets it
// step by step: msccl_interpreter.h:66-205).  For small calls the interpretation, not the bytes,
// is the cost: a one-shot schedule waits on a receive, publishes a flag, wakes a reduce thread
// block that re-reads the received copies from scratch and copies the result back.  When the
// program's RESULT on every rank is, for every chunk c, a left fold of all ranks' input chunk c
// in one fixed order per rank,
//     out_r[c] = x_{o_r(0)}[c] (+) x_{o_r(1)}[c] (+) ... (+) x_{o_r(n-1)}[c],
// the same values come out of one hop: every rank sends its input to every peer and folds the
// n inputs in the order o_r (the flat tree's fold kernel, with o_r as its order table).
//
// This file decides that, symbolically: it runs every rank's program (the XML loaded once per
// rank, as each rank loads it) on chunk-level expressions instead of data, with the reference's
// semantics for the LL protocol:
//   s / r / rcs            move values through the (channel, sender, receiver) FIFO, in order;
//   rrs / rrc / rrcs       fn(peer, local)                               (prims_ll.h:282-287)
//   re                     acc = d; acc = fn(acc, s_i) in reduction-table order
//                          (prims_ll.h:347-362; the small path o = fn(s_i, o),
//                          msccl_interpreter.h:157-170, is the same fold)
//   cpy                    copy
//   dependencies           (tb, step) is satisfied once tb published a flag >= step
//                          (msccl_interpreter.h:121-140,198-201), steps counted as the
//                          interpreter counts them (fused deps and reductions advance the count)
//   ra / unknown types     not lowered (the reference ends the thread block there)
// Expressions are hash-consed with fn(a, b) == fn(b, a): every op the lowering admits (Sum, Prod,
// Max, Min) is commutative per element in this runtime's arithmetic (IEEE add / mul, the fp16
// clamp, bf16 RNE of the exact result, integer wrap; the flat tree rests on the same fact,
// DESIGN.md §8), so a rank's result is then bit for bit the fold kernel's.  Anything else (a
// schedule that deadlocks, leaves FIFO messages, reads an uninitialised chunk into the result,
// folds chunks in a tree shape or in orders that differ between chunks of one rank) is not
// lowered.
#include <stdio.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "comm.h"
#include "debug.h"
#include "lower.h"

namespace msccl {

namespace {

struct Expr {
  int a, b;  // children (a < b) of fn; leaves have a = -1 and b = rank * nChunks + chunk
};

class Exprs {
 public:
  int leaf(int rank, int chunk, int nChunks) {
    const int key = rank * nChunks + chunk;
    auto it = leaves_.find(key);
    if (it != leaves_.end()) return it->second;
    nodes_.push_back({-1, key});
    creator_.push_back(rank);
    return leaves_[key] = (int)nodes_.size() - 1;
  }
  // fn(x, y) computed by a transfer of `rank` (the first rank to compute a value creates it)
  int op(int x, int y, int rank) {
    if (x < 0 || y < 0) return kUndef;  // an uninitialised chunk poisons the result
    const std::pair<int, int> k = x < y ? std::make_pair(x, y) : std::make_pair(y, x);
    auto it = ops_.find(k);
    if (it != ops_.end()) return it->second;
    nodes_.push_back({k.first, k.second});
    creator_.push_back(rank);
    return ops_[k] = (int)nodes_.size() - 1;
  }
  const Expr& at(int i) const { return nodes_[i]; }
  int creator(int i) const { return creator_[i]; }
  static constexpr int kUndef = -1;

 private:
  std::vector<Expr> nodes_;
  std::vector<int> creator_;
  std::map<int, int> leaves_;
  std::map<std::pair<int, int>, int> ops_;
};

struct TbState {
  size_t pc = 0;      // next transfer
  int step = 0;       // the interpreter's XML step counter
  int published = -1;
};

}  // namespace

// Runs every rank's program on chunk expressions (the semantics in the header comment; `re` in the
// protocol's order: LL / LL128 acc = d, acc = fn(acc, s_i) (prims_ll.h:347-362); Simple
// acc = s_0, acc = fn(acc, s_i), then fn(acc, d) (prims_simple.h:258-263, the big-call path)).
// inB[r] holds leaf(r, c) for c < cin, outB[r] cout undefined chunks (the output aliases the input
// of an in-place AllReduce).  Returns "" or why the schedule cannot be followed.
static std::string symRun(const std::vector<Algorithm>& byRank, int cin, int cout, bool simpleOrder, Exprs& ex,
                          std::vector<std::vector<int>>& inB, std::vector<std::vector<int>>& outB) {
  const int n = (int)byRank.size();
  std::vector<std::vector<int>> scrB(n);
  inB.assign(n, {});
  outB.assign(n, {});
  for (int r = 0; r < n; r++) {
    const Algorithm& a = byRank[r];
    inB[r].assign(std::max(cin, a.nInputChunks), Exprs::kUndef);
    for (int c = 0; c < (int)inB[r].size(); c++) inB[r][c] = c < cin ? ex.leaf(r, c, cin) : Exprs::kUndef;
    if (!a.inPlace) outB[r].assign(std::max(cout, a.nOutputChunks), Exprs::kUndef);
    scrB[r].assign(std::max(0, a.nScratchChunks), Exprs::kUndef);
  }
  auto buf = [&](int r, int id) -> std::vector<int>* {
    if (id == kInput) return &inB[r];
    if (id == kOutput) return byRank[r].inPlace ? &inB[r] : &outB[r];
    if (id == kScratch) return &scrB[r];
    return nullptr;
  };
  // FIFO of messages per (channel, sender, receiver)
  std::map<std::tuple<int, int, int>, std::vector<std::vector<int>>> fifo;
  std::vector<std::vector<TbState>> st(n);
  for (int r = 0; r < n; r++) st[r].assign(byRank[r].nBlocks, TbState());
  bool progress = true;
  size_t guard = 0;
  while (progress) {
    progress = false;
    for (int r = 0; r < n; r++) {
      const Algorithm& a = byRank[r];
      for (int b = 0; b < a.nBlocks; b++) {
        const ThreadBlock& tb = a.tbs[b];
        TbState& s = st[r][b];
        while (s.pc < tb.transfers.size()) {
          if (++guard > (size_t)1 << 24) return "schedule too large to analyse";
          const Transfer& t = tb.transfers[s.pc];
          bool ready = true;
          for (int d = 0; d < t.numDeps && ready; d++) {
            const int db = tb.depBid[t.depPtr + d], ds = tb.depStep[t.depPtr + d];
            if (db < 0 || db >= a.nBlocks) return "dependency on a missing thread block";
            ready = st[r][db].published >= ds;
          }
          const bool recv = t.type == kRecv || t.type == kRecvCopySend || t.type == kRecvReduceSend ||
                            t.type == kRecvReduceCopy || t.type == kRecvReduceCopySend;
          const bool send = t.type == kSend || t.type == kRecvCopySend || t.type == kRecvReduceSend ||
                            t.type == kRecvReduceCopySend;
          std::vector<std::vector<int>>* in = nullptr;
          if (ready && recv) {
            if (tb.recvpeer < 0) return "receive without a peer";
            in = &fifo[std::make_tuple((int)tb.channel, (int)tb.recvpeer, r)];
            ready = !in->empty();
          }
          if (!ready) break;
          if (send && tb.sendpeer < 0) return "send without a peer";
          const int cnt = t.count;
          std::vector<int>* src = buf(r, t.srcbuf);
          std::vector<int>* dst = buf(r, t.dstbuf);
          auto rd = [&](std::vector<int>* v, int off) -> int {
            if (v == nullptr || off < 0 || off >= (int)v->size()) return Exprs::kUndef;
            return (*v)[off];
          };
          auto wr = [&](std::vector<int>* v, int off, int x) -> bool {
            if (v == nullptr || off < 0 || off >= (int)v->size()) return false;
            (*v)[off] = x;
            return true;
          };
          std::vector<int> msg;
          if (recv) {
            msg = in->front();
            in->erase(in->begin());
            if ((int)msg.size() != cnt) return "receive count differs from the matching send";
          }
          std::vector<int> outMsg;
          switch (t.type) {
            case kSend:
              for (int c = 0; c < cnt; c++) outMsg.push_back(rd(src, t.srcoff + c));
              break;
            case kRecv:
              for (int c = 0; c < cnt; c++)
                if (!wr(dst, t.dstoff + c, msg[c])) return "receive into a missing chunk";
              break;
            case kRecvCopySend:
              for (int c = 0; c < cnt; c++)
                if (!wr(dst, t.dstoff + c, msg[c])) return "receive into a missing chunk";
              outMsg = msg;
              break;
            case kRecvReduceSend:
            case kRecvReduceCopy:
            case kRecvReduceCopySend:
              for (int c = 0; c < cnt; c++) {
                const int v = ex.op(msg[c], rd(src, t.srcoff + c), r);  // fn(peer, local) == fn(local, peer)
                if (t.type != kRecvReduceSend && !wr(dst, t.dstoff + c, v)) return "write to a missing chunk";
                if (t.type != kRecvReduceCopy) outMsg.push_back(v);
              }
              break;
            case kLocalCopy: {
              std::vector<int> v;
              for (int c = 0; c < cnt; c++) v.push_back(rd(src, t.srcoff + c));
              for (int c = 0; c < cnt; c++)
                if (!wr(dst, t.dstoff + c, v[c])) return "copy to a missing chunk";
              break;
            }
            case kReduce:
              for (int c = 0; c < cnt; c++) {
                int acc;
                if (simpleOrder) {
                  acc = rd(src, tb.redSrcOff[t.redPtr] + c);
                  for (int j = 1; j < t.numReds; j++) acc = ex.op(acc, rd(src, tb.redSrcOff[t.redPtr + j] + c), r);
                  acc = ex.op(acc, rd(dst, t.dstoff + c), r);
                } else {
                  acc = rd(dst, t.dstoff + c);
                  for (int j = 0; j < t.numReds; j++) acc = ex.op(acc, rd(src, tb.redSrcOff[t.redPtr + j] + c), r);
                }
                if (!wr(dst, t.dstoff + c, acc)) return "reduce into a missing chunk";
              }
              break;
            default:
              return "transfer type without a lowering (res-add or unknown)";
          }
          if (send) fifo[std::make_tuple((int)tb.channel, r, (int)tb.sendpeer)].push_back(outMsg);
          if (t.numDeps > 0) s.step += t.numDeps - 1;
          if (t.type == kReduce) s.step += t.numReds - 1;
          if (t.hasDep) s.published = s.step;
          s.step++;
          s.pc++;
          progress = true;
        }
      }
    }
  }
  for (int r = 0; r < n; r++)
    for (int b = 0; b < byRank[r].nBlocks; b++)
      if (st[r][b].pc < byRank[r].tbs[b].transfers.size()) return "schedule does not complete";
  for (auto& kv : fifo)
    if (!kv.second.empty()) return "unconsumed FIFO messages";
  for (int r = 0; r < n; r++)
    if (!byRank[r].inPlace)
      for (int c = 0; c < cin; c++)
        if (inB[r][c] != ex.leaf(r, c, cin)) return "an out-of-place schedule writes its input";
  return "";
}

// The ranks a result expression folds, innermost first: a left fold over leaves, each of them
// leaf(q, want) of input-chunk index `want` (cin chunks per rank), every rank once.
static std::string foldRanks(const Exprs& ex, int e, int want, int cin, int n, std::vector<int>* ranks) {
  std::vector<int> ord;  // leaf keys, outermost fold first
  if (e < 0) return "a result chunk is not a fold of the inputs";
  while (ex.at(e).a >= 0) {
    const Expr& x = ex.at(e);
    const bool la = ex.at(x.a).a < 0, lb = ex.at(x.b).a < 0;
    if (la && lb) {
      // the innermost fn(x_p, x_q): commutative, so the fold may start with either
      int p = ex.at(x.a).b, q = ex.at(x.b).b;
      if (p > q) std::swap(p, q);
      ord.push_back(q);
      ord.push_back(p);
      e = -1;
      break;
    }
    if (!la && !lb) return "a result chunk folds partial results in a tree shape";
    ord.push_back(la ? ex.at(x.a).b : ex.at(x.b).b);
    e = la ? x.b : x.a;
  }
  if (e >= 0) ord.push_back(ex.at(e).b);  // a lone leaf (no fold)
  ranks->clear();
  std::vector<bool> seen(n, false);
  for (auto it = ord.rbegin(); it != ord.rend(); ++it) {
    const int q = *it / cin, cc = *it % cin;
    if (cc != want || seen[q]) return "a result chunk is not a fold of every rank's same chunk";
    seen[q] = true;
    ranks->push_back(q);
  }
  if ((int)ranks->size() != n) return "a result chunk misses a rank";
  return "";
}

// classes of chunks whose orders (per rank) agree: ordOf[c][r] -> chunkClass, order
static void classesOf(const std::vector<std::vector<std::vector<int>>>& ordOf, std::vector<int>* chunkClass,
                      std::vector<std::vector<std::vector<int>>>* order) {
  chunkClass->assign(ordOf.size(), -1);
  order->clear();
  for (size_t c = 0; c < ordOf.size(); c++) {
    for (size_t k = 0; k < order->size() && (*chunkClass)[c] < 0; k++)
      if ((*order)[k] == ordOf[c]) (*chunkClass)[c] = (int)k;
    if ((*chunkClass)[c] < 0) {
      (*chunkClass)[c] = (int)order->size();
      order->push_back(ordOf[c]);
    }
  }
}

FoldLowering analyzeFoldLowering(const std::vector<Algorithm>& byRank) {
  FoldLowering out;
  const int n = (int)byRank.size();
  auto fail = [&](const std::string& why) {
    out.ok = false;
    out.why = why;
    out.order.clear();
    out.chunkClass.clear();
    return out;
  };
  if (n < 2 || n > kMaxReduceFusion) return fail("ranks outside 2..16");
  const Algorithm& a0 = byRank[0];
  const int C = a0.nchunksPerLoop;
  if (C <= 0) return fail("no chunks");
  for (const Algorithm& a : byRank) {
    if (!a.valid || a.coll != kAllReduce) return fail("not a valid AllReduce schedule");
    if (a.proto != kProtoLL) return fail("protocol is not LL");
    if (a.nchunksPerLoop != C || a.inPlace != a0.inPlace) return fail("ranks disagree on the loop shape");
  }
  Exprs ex;
  std::vector<std::vector<int>> inB, outB;
  const std::string why = symRun(byRank, C, C, false, ex, inB, outB);
  if (!why.empty()) return fail(why);
  // every result chunk: a left fold of all ranks' same chunk; orders per (chunk, rank)
  std::vector<std::vector<std::vector<int>>> ordOf(C, std::vector<std::vector<int>>(n));
  for (int r = 0; r < n; r++) {
    const std::vector<int>& res = byRank[r].inPlace ? inB[r] : outB[r];
    for (int c = 0; c < C; c++) {
      const std::string w = foldRanks(ex, res[c], c, C, n, &ordOf[c][r]);
      if (!w.empty()) return fail(w);
    }
  }
  classesOf(ordOf, &out.chunkClass, &out.order);
  if ((int)out.order.size() > kMaxFoldClasses) return fail("more fold orders than the fold kernel holds");
  if (out.order.size() > 1 && C > kMaxFoldChunks) return fail("more chunks than the fold kernel's class map holds");
  out.ok = true;
  // the two-phase form: every rank's chunk c is the same value (hash-consed: the same node), and
  // its creator owns it; every rank must own C / n chunks (the kernel deals the owned chunks of all
  // ranks out to its workgroups in lockstep)
  auto notTwoPhase = [&](const std::string& w) {
    out.twoPhase = false;
    out.whyNotTwoPhase = w;
    out.owner.clear();
    return out;
  };
  if (C > kMaxFoldChunks) return notTwoPhase("more chunks than the two-phase kernel's tables hold");
  if (C % n != 0) return notTwoPhase("the chunks do not divide over the ranks");
  out.owner.assign(C, -1);
  std::vector<int> owned(n, 0);
  for (int c = 0; c < C; c++) {
    const int e = byRank[0].inPlace ? inB[0][c] : outB[0][c];
    for (int r = 1; r < n; r++)
      if ((byRank[r].inPlace ? inB[r][c] : outB[r][c]) != e)
        return notTwoPhase("ranks hold different folds of a chunk (a one-shot schedule)");
    const int q = ex.creator(e);
    out.owner[c] = q;
    owned[q]++;
  }
  for (int q = 0; q < n; q++)
    if (owned[q] != C / n) return notTwoPhase("ranks own different numbers of chunks");
  out.twoPhase = true;
  return out;
}

DirectLowering analyzeDirectLowering(const std::vector<Algorithm>& byRank) {
  DirectLowering out;
  const int n = (int)byRank.size();
  auto fail = [&](const std::string& why) {
    out = DirectLowering();
    out.why = why;
    return out;
  };
  if (n < 2 || n > kMaxReduceFusion) return fail("ranks outside 2..16");
  const Algorithm& a0 = byRank[0];
  const int C = a0.nchunksPerLoop;
  if (C <= 0 || C % n != 0) return fail("no chunks, or chunks that do not divide over the ranks");
  const int coll = a0.coll;
  if (coll != kAllReduce && coll != kReduceScatter && coll != kAllGather)
    return fail("not an AllReduce, ReduceScatter or AllGather");
  for (const Algorithm& a : byRank) {
    if (!a.valid || a.coll != coll) return fail("ranks disagree on the collective");
    if (a.proto != kProtoSimple) return fail("protocol is not Simple");
    if (a.nchunksPerLoop != C || a.inPlace != a0.inPlace) return fail("ranks disagree on the loop shape");
    if (coll != kAllReduce && a.inPlace) return fail("an in-place ReduceScatter / AllGather schedule");
  }
  // chunks per rank buffer: the AllGather's input is one rank's block, the ReduceScatter's output
  const int cin = coll == kAllGather ? C / n : C, cout = coll == kReduceScatter ? C / n : C;
  Exprs ex;
  std::vector<std::vector<int>> inB, outB;
  const std::string why = symRun(byRank, cin, cout, true, ex, inB, outB);
  if (!why.empty()) return fail(why);
  out.coll = coll;
  if (coll == kAllGather) {
    // the AllGather's definition: output chunk c of every rank is rank c / (C / n)'s input chunk
    for (int r = 0; r < n; r++)
      for (int c = 0; c < C; c++)
        if (outB[r][c] != ex.leaf(c / cin, c % cin, cin)) return fail("an output chunk is not its rank's input chunk");
    out.ok = true;
    return out;
  }
  // ReduceScatter: rank r's output chunk c folds every rank's input chunk r * C / n + c; AllReduce:
  // every rank's chunk c folds every rank's chunk c, and every rank holds the same value (one rank
  // computes it for all: the direct kernel's owner)
  std::vector<std::vector<std::vector<int>>> ordOf(cout, std::vector<std::vector<int>>(n));
  for (int r = 0; r < n; r++) {
    const std::vector<int>& res = byRank[r].inPlace ? inB[r] : outB[r];
    for (int c = 0; c < cout; c++) {
      const int want = coll == kReduceScatter ? r * cout + c : c;
      const std::string w = foldRanks(ex, res[c], want, cin, n, &ordOf[c][r]);
      if (!w.empty()) return fail(w);
      if (coll == kAllReduce && res[c] != (byRank[0].inPlace ? inB[0][c] : outB[0][c]))
        return fail("ranks hold different folds of a chunk");
    }
  }
  classesOf(ordOf, &out.chunkClass, &out.order);
  if ((int)out.order.size() > kMaxDirectClasses) return fail("more fold orders than the direct kernel holds");
  if (cout > kMaxFoldChunks) return fail("more chunks than the direct kernel's class map holds");
  out.ok = true;
  return out;
}

bool lowerOffered() {
  // NPKit and the full trace (MSCCL_AMD_TRACE=1) record the schedule's own primitives
  // (msccl_interpreter.h's placement): a rank with either on offers no lowering, and the init
  // allgather then keeps the interpreter on every rank, so a traced schedule runs as written
  return envInt("MSCCL_AMD_NPKIT", 0) <= 0 && envInt("MSCCL_AMD_TRACE", 0) != 1;
}

FoldLowering lowerScheduleFile(const std::string& path, int nRanks) {
  // the file's text and the rank count are the key: a path may be rewritten between
  // communicators of one process (a bench writes its tier files again under the same names)
  std::string text;
  if (FILE* f = fopen(path.c_str(), "rb")) {
    char buf[65536];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, got);
    fclose(f);
  }
  static std::mutex mu;
  static std::map<std::pair<std::string, int>, FoldLowering> cache;
  const auto key = std::make_pair(text, nRanks);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  FoldLowering fl;
  std::vector<Algorithm> byRank(nRanks);
  for (int r = 0; r < nRanks; r++)
    if (loadAlgoFromXml(path.c_str(), &byRank[r], kMaxChannels, r, nRanks) != 0) {
      fl.why = "the schedule does not load for rank " + std::to_string(r);
      return fl;
    }
  fl = analyzeFoldLowering(byRank);
  std::lock_guard<std::mutex> g(mu);
  if (cache.size() > 256) cache.clear();  // a bound for long-lived processes
  cache.emplace(key, fl);
  return fl;
}

DirectLowering directScheduleFile(const std::string& path, int nRanks) {
  std::string text;
  if (FILE* f = fopen(path.c_str(), "rb")) {
    char buf[65536];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, got);
    fclose(f);
  }
  static std::mutex mu;
  static std::map<std::pair<std::string, int>, DirectLowering> cache;
  const auto key = std::make_pair(text, nRanks);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  DirectLowering dl;
  std::vector<Algorithm> byRank(nRanks);
  for (int r = 0; r < nRanks; r++)
    if (loadAlgoFromXml(path.c_str(), &byRank[r], kMaxChannels, r, nRanks) != 0) {
      dl.why = "the schedule does not load for rank " + std::to_string(r);
      return dl;
    }
  dl = analyzeDirectLowering(byRank);
  std::lock_guard<std::mutex> g(mu);
  if (cache.size() > 256) cache.clear();
  cache.emplace(key, dl);
  return dl;
}

}  // namespace msccl
