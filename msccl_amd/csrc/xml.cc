// MSCCL XML schedule loader.
//
// Accept/reject semantics restate the reference loader:
//   tokenizer        graph/xml.cc:20-211  (xmlGetValue / xmlGetToken / xmlSkipComment /
//                                          xmlGetNode / xmlLoadSub)
//   rank filtering   graph/xml.cc:850-893 (only <gpu id==rank> children are retained)
//   attribute reads  graph/xml.h:67-120   (strtol(.., 0) integer parsing)
//   algo building    graph/topo.cc:759-1193 (validation, re-chain fusion, nop dependency
//                                          packing, contiguous tb ids)
//   file lists       graph/topo.cc:1195-1284 (MSCCL_XML_FILES, MSCCL_CONFIG)
// The whole file is read into memory once instead of fread(1) per character.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <sstream>

#include "algo.h"
#include "debug.h"

namespace msccl {

namespace {

constexpr int kMaxStrLen = 255;     // xml.h:16
constexpr int kMaxAttrCount = 16;   // xml.h:17
constexpr int kMaxSubs = 1024;      // xml.h:18
constexpr int kMaxNodes = 1 << 12;  // xml.h:19

enum NodeType { kNone = 0, kOpen = 1, kClose = 2, kSingle = 3 };

// ncclResult_t values
constexpr int kInternal = 3, kInvalidUsage = 5, kSystem = 2;

struct Node {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;  // first kMaxAttrCount kept
  int type = kNone;
  std::vector<Node*> subs;
};

struct Reader {
  std::string buf;
  size_t pos = 0;
  bool get(char* c) {
    if (pos >= buf.size()) return false;
    *c = buf[pos++];
    return true;
  }
};

struct Doc {
  std::vector<std::unique_ptr<Node>> nodes;  // retained nodes (xml->nodes[0..maxIndex))
  int maxIndex = 0;
};

int getChar(Reader& r, char* c) {
  if (!r.get(c)) { WARN("XML Parse : Unexpected EOF"); return kInternal; }
  return 0;
}

// xml.cc:28-55 — value must start with a quote; it ends at the next '"'
int getValue(Reader& r, std::string* value, char* last) {
  char c;
  MSCCLCHECK(getChar(r, &c));
  if (c != '"' && c != '\'') { WARN("XML Parse : Expected (double) quote."); return kInternal; }
  value->clear();
  while (true) {
    MSCCLCHECK(getChar(r, &c));
    if (c == '"') break;
    value->push_back(c);
    // The reference writes into a MAX_STR_LEN+1 buffer without a bound; reject instead.
    if ((int)value->size() > kMaxStrLen) { WARN("XML Parse : value too long"); return kInternal; }
  }
  return getChar(r, last);
}

// xml.cc:57-80 — reads a name up to ' ', '>', '/', '\n', '\r' or '='
int getToken(Reader& r, std::string* name, std::string* value, char* last) {
  name->clear();
  char c;
  int o = 0;
  do {
    MSCCLCHECK(getChar(r, &c));
    if (c == '=') {
      if (value == nullptr) { WARN("XML Parse : Unexpected value with name %s", name->c_str()); return kInternal; }
      return getValue(r, value, last);
    }
    name->push_back(c);
    if (o == kMaxStrLen - 1) { WARN("Error : name too long (max %d)", kMaxStrLen); return kInternal; }
    o++;
  } while (c != ' ' && c != '>' && c != '/' && c != '\n' && c != '\r');
  name->pop_back();  // drop the terminator
  *last = c;
  return 0;
}

// xml.cc:84-104 — skip until "-->" (the trailing chars already read count)
int skipComment(Reader& r, const std::string& start, char next) {
  char end[4] = "...";
  auto push = [&](char ch) { end[0] = end[1]; end[1] = end[2]; end[2] = ch; };
  for (char ch : start) push(ch);
  push(next);
  while (strcmp(end, "-->") != 0) {
    char c;
    if (!r.get(&c)) { WARN("XML Parse error : unterminated comment"); return kInternal; }
    push(c);
  }
  return 0;
}

// xml.cc:106-155
int getNode(Reader& r, Node* node) {
  node->type = kNone;
  node->name.clear();
  node->attrs.clear();
  node->subs.clear();
  char c = ' ';
  while (c == ' ' || c == '\n' || c == '\r') {
    if (!r.get(&c)) return 0;
  }
  if (c != '<') { WARN("XML Parse error : expecting '<', got '%c'", c); return kInternal; }
  MSCCLCHECK(getToken(r, &node->name, nullptr, &c));
  if (node->name.compare(0, 3, "!--") == 0) {
    MSCCLCHECK(skipComment(r, node->name.substr(3), c));
    return getNode(r, node);
  }
  if (node->name.empty() && c == '/') {
    node->type = kClose;
    MSCCLCHECK(getToken(r, &node->name, nullptr, &c));
    if (c != '>') { WARN("XML Parse error : unexpected trailing %c in closing tag %s", c, node->name.c_str()); return kInternal; }
    return 0;
  }
  node->type = kOpen;
  while (c == ' ') {
    std::string k, v;
    MSCCLCHECK(getToken(r, &k, &v, &c));
    // Attributes past MAX_ATTR_COUNT are consumed but dropped (xml.cc:136-140).
    if ((int)node->attrs.size() < kMaxAttrCount) node->attrs.emplace_back(k, v);
  }
  if (c == '/') {
    node->type = kSingle;
    std::string s;
    MSCCLCHECK(getToken(r, &s, nullptr, &c));
  }
  if (c != '>') { WARN("XML Parse : expected >, got '%c'", c); return kInternal; }
  return 0;
}

// Handlers mirror the reference's nested handler tables (xml.cc:850-893).
enum Handler { kHNone, kHAlgo, kHGpu, kHTb, kHStep, kHMsccl, kHLoad };

struct Loader {
  Reader r;
  Doc doc;
  int myrank = 0;
  bool configMode = false;

  const char* handlerName(Handler h) {
    switch (h) {
      case kHAlgo: return "algo";
      case kHGpu: return "gpu";
      case kHTb: return "tb";
      case kHStep: return "step";
      case kHMsccl: return "msccl_algos";
      case kHLoad: return "load";
      default: return "";
    }
  }

  // Skip a subtree.  In the reference an unknown element is parsed into the
  // same node slot as its parent, so any closing tag ends the level and
  // EOF inside it is an error (xml.cc:170-187,206-208).
  int skipSub(int headType) {
    if (headType == kSingle) return 0;
    Node tmp;
    while (true) {
      MSCCLCHECK(getNode(r, &tmp));
      if (tmp.type == kNone) { WARN("XML Parse : unterminated element"); return kInternal; }
      if (tmp.type == kClose) return 0;
      INFO(kSubGraph, "Ignoring element %s", tmp.name.c_str());
      MSCCLCHECK(skipSub(tmp.type));
    }
  }

  int handle(Handler h, Node* node);

  // xml.cc:168-211 with a handler list (zero or one handler in every MSCCL table)
  int loadSub(Node* head, Handler handler) {
    if (head && head->type == kSingle) return 0;
    while (true) {
      if (doc.maxIndex == kMaxNodes) { WARN("Error : XML parser is limited to %d nodes", kMaxNodes); return kInternal; }
      auto node = std::make_unique<Node>();
      MSCCLCHECK(getNode(r, node.get()));
      if (node->type == kNone) {
        if (head) { WARN("XML Parse : unterminated %s", head->name.c_str()); return kInternal; }
        return 0;
      }
      if (head && node->type == kClose) {
        if (node->name != head->name) { WARN("XML Mismatch : %s / %s", head->name.c_str(), node->name.c_str()); return kInternal; }
        return 0;
      }
      if (handler != kHNone && node->name == handlerName(handler)) {
        if (head) {
          if ((int)head->subs.size() == kMaxSubs) { WARN("XML Parse : too many children of %s", head->name.c_str()); return kInternal; }
          head->subs.push_back(node.get());
        }
        Node* n = node.get();
        doc.nodes.push_back(std::move(node));
        doc.maxIndex++;
        MSCCLCHECK(handle(handler, n));
      } else {
        if (handler != kHNone) INFO(kSubGraph, "Ignoring element %s", node->name.c_str());
        MSCCLCHECK(skipSub(node->type));
      }
    }
  }

  Node* findTag(const char* name) {
    for (auto& n : doc.nodes)
      if (n->name == name) return n.get();
    return nullptr;
  }
};

const std::string* getAttr(const Node* n, const char* key) {
  for (auto& kv : n->attrs)
    if (kv.first == key) return &kv.second;
  return nullptr;
}
int getAttrStr(const Node* n, const char* key, const char** v) {
  const std::string* s = getAttr(n, key);
  if (!s) { WARN("Attribute %s of node %s not found", key, n->name.c_str()); return kInternal; }
  *v = s->c_str();
  return 0;
}
int getAttrInt(const Node* n, const char* key, int* v) {
  const char* s;
  MSCCLCHECK(getAttrStr(n, key, &s));
  *v = (int)strtol(s, nullptr, 0);
  return 0;
}
int getAttrInt64(const Node* n, const char* key, int64_t* v) {
  const char* s;
  MSCCLCHECK(getAttrStr(n, key, &s));
  *v = strtoll(s, nullptr, 0);
  return 0;
}

int Loader::handle(Handler h, Node* node) {
  switch (h) {
    case kHAlgo: return loadSub(node, kHGpu);
    case kHGpu: {
      int id;
      MSCCLCHECK(getAttrInt(node, "id", &id));
      if (id == myrank) return loadSub(node, kHTb);
      return loadSub(node, kHNone);
    }
    case kHTb: return loadSub(node, kHStep);
    case kHStep:
      // The reference recurses with a NULL handler table here: a <step> that is
      // not self-closing dereferences NULL (xml.cc:846-849).  Reject it.
      if (node->type != kSingle) { WARN("MSCCL: <step> must be a single (self-closing) element"); return kInternal; }
      return 0;
    case kHMsccl: return loadSub(node, kHLoad);
    case kHLoad: return loadSub(node, kHNone);
    default: return 0;
  }
}

int readFile(const char* path, std::string* out) {
  FILE* f = fopen(path, "r");
  if (!f) { WARN("Could not open XML MSCCL graph file %s : %s", path, strerror(errno)); return kSystem; }
  char tmp[65536];
  size_t n;
  while ((n = fread(tmp, 1, sizeof(tmp), f)) > 0) out->append(tmp, n);
  fclose(f);
  return 0;
}

int bufferType(const char* s, uint8_t* out) {  // topo.cc:711-723
  if (!strcmp(s, "i")) *out = kInput;
  else if (!strcmp(s, "o")) *out = kOutput;
  else if (!strcmp(s, "s")) *out = kScratch;
  else { WARN("type of buffer is not supported: %s", s); return kInvalidUsage; }
  return 0;
}

int checkBounds(int buf, int off, int nIn, int nOut, int nScr) {  // topo.cc:725-743
  int lim = buf == kInput ? nIn : buf == kOutput ? nOut : nScr;
  const char* nm = buf == kInput ? "input" : buf == kOutput ? "output" : "scratch";
  if (off < -1 || off >= lim) {
    WARN("Incorrect offset set for %s buffer: offset: %d maximum allowed: %d", nm, off, lim);
    return kInvalidUsage;
  }
  return 0;
}

}  // namespace

int protoFromStr(const char* p, int* id) {  // topo.cc:745-757
  if (!p) { WARN("MSCCL: protocol is missing"); return kInvalidUsage; }
  if (!strcmp(p, "Simple")) *id = kProtoSimple;
  else if (!strcmp(p, "LL128")) *id = kProtoLL128;
  else if (!strcmp(p, "LL")) *id = kProtoLL;
  else { WARN("MSCCL: protocol %s is not supported.", p); return kInvalidUsage; }
  return 0;
}

// topo.cc:759-1193
int loadAlgoFromXml(const char* path, Algorithm* algo, int maxNChannels, int rank, int nRanks) {
  INFO(kSubInit, "MSCCL: Parsing algorithm %s", path);
  Loader L;
  L.myrank = rank;
  MSCCLCHECK(readFile(path, &L.r.buf));
  MSCCLCHECK(L.loadSub(nullptr, kHAlgo));

  *algo = Algorithm();
  algo->path = path;
  algo->valid = false;
  Node* top = L.findTag("algo");
  if (!top) { WARN("MSCCL: no <algo> element in %s", path); return kInternal; }
  const char* name;
  MSCCLCHECK(getAttrStr(top, "name", &name));
  algo->name = std::string(name).substr(0, 63);  // MSCCL_MAX_ALGO_NAME

  int ngpus;
  MSCCLCHECK(getAttrInt(top, "ngpus", &ngpus));
  if (nRanks != ngpus) {
    WARN("MSCCL: ngpus set in the MSCCL algo (%d) doesn't match the communicator ngpus (%d)", ngpus, nRanks);
    return kInvalidUsage;
  }
  algo->ngpus = ngpus;
  int ncpl, nch;
  MSCCLCHECK(getAttrInt(top, "nchunksperloop", &ncpl));
  MSCCLCHECK(getAttrInt(top, "nchannels", &nch));
  const char* proto;
  MSCCLCHECK(getAttrStr(top, "proto", &proto));
  MSCCLCHECK(protoFromStr(proto, &algo->proto));

  int64_t minBytes = 0, maxBytes = (int64_t)1 << 27;
  if (getAttr(top, "minBytes")) MSCCLCHECK(getAttrInt64(top, "minBytes", &minBytes));
  if (getAttr(top, "maxBytes")) MSCCLCHECK(getAttrInt64(top, "maxBytes", &maxBytes));
  if (minBytes > maxBytes) { WARN("MSCCL: minBytes cannot be greater than maxBytes."); return kInvalidUsage; }
  if (minBytes < 0) { WARN("MSCCL: minBytes cannot be negative."); return kInvalidUsage; }
  if (maxBytes < 0) { WARN("MSCCL: maxBytes cannot be negative."); return kInvalidUsage; }
  algo->minBytes = minBytes;
  algo->maxBytes = maxBytes;

  const char* coll;
  MSCCLCHECK(getAttrStr(top, "coll", &coll));
  int inMul = 1, outMul = 1;
  if (!strcmp(coll, "allreduce")) algo->coll = kAllReduce;
  else if (!strcmp(coll, "allgather")) { algo->coll = kAllGather; inMul = nRanks; }
  else if (!strcmp(coll, "reduce")) algo->coll = kReduceColl;
  else if (!strcmp(coll, "broadcast")) algo->coll = kBroadcast;
  else if (!strcmp(coll, "alltoall")) algo->coll = kAllToAll;
  else if (!strcmp(coll, "reduce_scatter")) { algo->coll = kReduceScatter; outMul = nRanks; }
  else if (!strcmp(coll, "custom")) algo->coll = kCustom;
  else { WARN("MSCCL: collective type %s is not supported.", coll); return kInvalidUsage; }

  int inplace;
  MSCCLCHECK(getAttrInt(top, "inplace", &inplace));
  algo->inPlace = inplace ? 1 : 0;
  int nThreads = 0;
  if (getAttr(top, "nthreads")) {
    MSCCLCHECK(getAttrInt(top, "nthreads", &nThreads));
    if (nThreads % kRefWarp != 0) { WARN("MSCCL nthreads must be a multiplication of %d", kRefWarp); return kInvalidUsage; }
  }
  algo->nThreads = nThreads;
  if (nch > maxNChannels) WARN("MSCCL: number of desired channels (%d) is more than possible ones (%d)", nch, maxNChannels);
  algo->nChannels = nch;
  algo->nchunksPerLoop = ncpl;

  std::vector<ThreadBlock> tbs(kMaxTb);
  std::vector<int> blockExists(kMaxTb, 0);
  for (Node* node : top->subs) {
    if (node->name != "gpu") continue;
    int id, nScr, nIn, nOut;
    MSCCLCHECK(getAttrInt(node, "id", &id));
    if (id != rank) continue;
    MSCCLCHECK(getAttrInt(node, "i_chunks", &nIn));
    MSCCLCHECK(getAttrInt(node, "o_chunks", &nOut));
    MSCCLCHECK(getAttrInt(node, "s_chunks", &nScr));
    if (nScr < 0) { WARN("MSCCL: nScratchChunks must be not negative. nScratchChunks: %d", nScr); return kInvalidUsage; }
    if ((nIn > 0 && nIn * inMul != ncpl) || (nOut > 0 && nOut * outMul != ncpl)) {
      WARN("Inconsistency between i_chunks/o_chunks (%d/%d) and nchunksperloop (%d) for collective %s", nIn, nOut, ncpl, coll);
      return kInvalidUsage;
    }
    algo->nScratchChunks = nScr;
    algo->nInputChunks = nIn;
    algo->nOutputChunks = nOut;
    for (Node* tbn : node->subs) {
      if (tbn->name != "tb") continue;
      int bid, recvpeer, sendpeer, chan;
      MSCCLCHECK(getAttrInt(tbn, "id", &bid));
      MSCCLCHECK(getAttrInt(tbn, "recv", &recvpeer));
      MSCCLCHECK(getAttrInt(tbn, "send", &sendpeer));
      MSCCLCHECK(getAttrInt(tbn, "chan", &chan));
      if (bid < 0) { WARN("MSCCL: bid must be not negative. bid: %d", bid); return kInvalidUsage; }
      if (bid >= kMaxTb) { WARN("MSCCL: too many thread blocks are requested. Max thread blocks: %d", kMaxTb); return kInvalidUsage; }
      if (blockExists[bid]) { WARN("MSCCL: duplicate thread block id %d for MSCCL", bid); return kInvalidUsage; }
      blockExists[bid] = 1;
      if (recvpeer == id || sendpeer == id) { WARN("MSCCL: peer (%d,%d) and gpu id (%d) must be different", recvpeer, sendpeer, id); return kInvalidUsage; }
      ThreadBlock& tb = tbs[bid];
      tb = ThreadBlock();
      tb.exists = true;
      if (recvpeer < -1 || sendpeer < -1) { WARN("MSCCL: wrong recvpeer (%d) or sendpeer (%d) in threadblock %d on gpu %d", recvpeer, sendpeer, bid, id); return kInvalidUsage; }
      if (recvpeer >= ngpus || sendpeer >= ngpus) { WARN("MSCCL: recvpeer (%d) or sendpeer (%d) must be -1 or between 0 and ngpus (%d)", recvpeer, sendpeer, ngpus); return kInvalidUsage; }
      tb.recvpeer = recvpeer;
      tb.sendpeer = sendpeer;
      // The reference accepts chan == MAXCHANNELS (topo.cc:936, off by one) and
      // then indexes mscclChannels[32] out of bounds; reject it here.
      if (chan < 0 || chan >= kMaxChannels) { WARN("MSCCL: threadblock %d on GPU %d has an invalid channel %d", bid, id, chan); return kInvalidUsage; }
      tb.channel = (int8_t)chan;

      int numDeps = 0, oldDepPtr = 0;
      int oldRedDstBuf = -1, oldRedDstOff = -1, oldRedSrcBuf = -1;
      int numReds = 0, numTransfers = 0;
      tb.transfers.resize(kMaxSteps);
      tb.depBid.assign(kMaxSteps, 0);
      tb.depStep.assign(kMaxSteps, 0);
      tb.redSrcOff.assign(kMaxSteps, 0);
      for (Node* st : tbn->subs) {
        if (st->name != "step") continue;
        int s, srcoff, dstoff, depBid, depStep, hasDep, count;
        const char *srcbuf, *dstbuf, *type;
        MSCCLCHECK(getAttrInt(st, "s", &s));
        MSCCLCHECK(getAttrInt(st, "srcoff", &srcoff));
        MSCCLCHECK(getAttrStr(st, "srcbuf", &srcbuf));
        MSCCLCHECK(getAttrInt(st, "dstoff", &dstoff));
        MSCCLCHECK(getAttrStr(st, "dstbuf", &dstbuf));
        MSCCLCHECK(getAttrInt(st, "cnt", &count));
        MSCCLCHECK(getAttrStr(st, "type", &type));
        MSCCLCHECK(getAttrInt(st, "depid", &depBid));
        MSCCLCHECK(getAttrInt(st, "deps", &depStep));
        MSCCLCHECK(getAttrInt(st, "hasdep", &hasDep));
        if (s >= kMaxSteps) { WARN("MSCCL: too many steps are requested. Max number of steps: %d, requested: %d", kMaxSteps, s + 1); return kInternal; }
        if (s < 0) { WARN("MSCCL: step must be positive: step %d", s); return kInternal; }

        int hasSend = 0, hasRecv = 0, checkSrc = 0, checkDst = 0, tt = -1;
        if (!strcmp(type, "s")) { tt = kSend; hasSend = 1; checkSrc = 1; }
        else if (!strcmp(type, "r")) { tt = kRecv; hasRecv = 1; checkDst = 1; }
        else if (!strcmp(type, "rcs")) { tt = kRecvCopySend; hasSend = hasRecv = 1; checkDst = 1; }
        else if (!strcmp(type, "rrs")) { tt = kRecvReduceSend; hasSend = hasRecv = 1; checkSrc = 1; }
        else if (!strcmp(type, "rrc")) { tt = kRecvReduceCopy; hasRecv = 1; }
        else if (!strcmp(type, "rrcs")) { tt = kRecvReduceCopySend; hasRecv = hasSend = 1; checkSrc = checkDst = 1; }
        else if (!strcmp(type, "cpy")) { tt = kLocalCopy; checkSrc = checkDst = 1; }
        else if (!strcmp(type, "re")) { tt = kReduce; checkSrc = checkDst = 1; }
        else if (!strcmp(type, "ra")) { tt = kResAdd; checkSrc = checkDst = 1; }
        else if (!strcmp(type, "nop")) { tt = -1; }
        else { WARN("MSCCL: type of transfer is not supported: %s", type); return kInternal; }

        if (depBid >= 0) {
          if (numDeps >= kMaxSteps) { WARN("MSCCL: too many dependences in threadblock %d", bid); return kInvalidUsage; }
          tb.depBid[numDeps] = (int16_t)depBid;
          tb.depStep[numDeps] = (int16_t)depStep;
          numDeps++;
        }
        uint8_t sb = 0, db = 0;
        MSCCLCHECK(bufferType(srcbuf, &sb));
        MSCCLCHECK(bufferType(dstbuf, &db));

        int continuation = 0;
        if (tt == kReduce) {
          if (oldRedDstBuf == db && oldRedDstOff == dstoff && oldRedSrcBuf == sb && depBid == -1) {
            numTransfers--;
            continuation = 1;
          } else {
            oldRedDstBuf = -1;
            oldRedDstOff = -1;
          }
        }
        if (tt == -1) continue;
        if (numTransfers >= kMaxSteps || numReds >= kMaxSteps) {
          WARN("MSCCL: too many steps in threadblock %d on GPU %d", bid, id);
          return kInvalidUsage;
        }

        Transfer& t = tb.transfers[numTransfers];
        t.type = (uint8_t)tt;
        t.srcoff = (int16_t)srcoff;
        t.srcbuf = sb;
        t.dstbuf = db;
        t.dstoff = (int16_t)dstoff;
        if (count < 0 || count >= kMaxCount) { WARN("MSCCL: count (%d) must be positive and less than %d", count, kMaxCount); return kInternal; }
        t.count = (uint8_t)count;
        if (hasSend && sendpeer < 0) { WARN("MSCCL: there is a send in threadblock %d on GPU %d without a sendpeer.", bid, id); return kInvalidUsage; }
        if (hasRecv && recvpeer < 0) { WARN("MSCCL: there is a recv in threadblock %d on GPU %d without a recvpeer.", bid, id); return kInvalidUsage; }
        if (checkSrc) MSCCLCHECK(checkBounds(t.srcbuf, t.srcoff, nIn, nOut, nScr));
        if (checkDst) MSCCLCHECK(checkBounds(t.dstbuf, t.dstoff, nIn, nOut, nScr));
        if (!continuation) {
          t.depPtr = (int16_t)oldDepPtr;
          t.numDeps = (int16_t)(numDeps - oldDepPtr);
          if (t.numDeps > 0 && depBid < 0) {
            WARN("MSCCL: when there is a chain of dependences, the last reduction must be a part of the first immediate instruction. Detected for GPU %d, threadblock %d, and step %d. XML will be ignored.", id, bid, s);
            return kInvalidUsage;
          }
          oldDepPtr = numDeps;
        }
        if (tt != kReduce) {
          oldRedDstBuf = oldRedDstOff = oldRedSrcBuf = -1;
        } else {
          if (oldRedDstBuf == -1) t.redPtr = (int16_t)numReds;
          tb.redSrcOff[numReds] = t.srcoff;
          numReds++;
          t.numReds = (int16_t)(numReds - t.redPtr);
          if (hasDep || numReds == kMaxReduceFusion) {
            oldRedDstBuf = oldRedDstOff = -1;
          } else {
            oldRedDstBuf = t.dstbuf;
            oldRedDstOff = t.dstoff;
            oldRedSrcBuf = t.srcbuf;
          }
          // The reference fuses past 16 sources when its per-tb counter is not
          // exactly 16 (topo.cc:1125) and then overflows srcs[17] in the kernel
          // (msccl_interpreter.h:175).  Reject such programs.
          if (t.numReds > kMaxReduceFusion) { WARN("MSCCL: reduction chain longer than %d in threadblock %d", kMaxReduceFusion, bid); return kInvalidUsage; }
        }
        if (hasDep != 0 && hasDep != 1) { WARN("MSCCL: has_dependence needs to be 0 or 1, but it was %d", hasDep); return kInternal; }
        t.hasDep = (int8_t)hasDep;
        numTransfers++;
        tb.nsteps = (uint16_t)numTransfers;
      }
      tb.transfers.resize(tb.nsteps);
      tb.depBid.resize(numDeps);
      tb.depStep.resize(numDeps);
      tb.redSrcOff.resize(numReds);
    }
    // topo.cc:1173-1185 — thread block ids must be contiguous from 0
    if (blockExists[0]) algo->nBlocks = 1;
    for (int i = 1; i < kMaxTb; i++) {
      if (blockExists[i] && !blockExists[i - 1]) { WARN("MSCCL: threadblock %d is missing", i); return kInvalidUsage; }
      if (blockExists[i]) algo->nBlocks = i + 1;
    }
  }
  tbs.resize(algo->nBlocks);
  algo->tbs = std::move(tbs);
  algo->valid = true;
  return 0;
}

// topo.cc:1195-1217 — ':'-separated list; failures are WARNed and skipped
int loadAlgosFromXmlFiles(const char* list, std::vector<Algorithm>* algos, int maxNChannels, int rank, int nRanks) {
  INFO(kSubEnv, "MSCCL_XML_FILES set by environment to %s", list);
  std::string s(list);
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(':', p);
    if (q == std::string::npos) q = s.size();
    std::string tok = s.substr(p, q - p);
    p = q + 1;
    if (tok.empty()) continue;  // strtok_r skips empty tokens
    if ((int)algos->size() == kMaxAlgos) {
      WARN("MSCCL: too many algorithms (%d) specified in environment variable MSCCL_XML_FILES. The rest will be ignored.", (int)algos->size());
      break;
    }
    Algorithm a;
    if (loadAlgoFromXml(tok.c_str(), &a, maxNChannels, rank, nRanks) == 0) {
      algos->push_back(std::move(a));
      INFO(kSubInit, "Parsed MSCCL Algorithm %s successfully.", tok.c_str());
    } else {
      WARN("MSCCL: algorithm %s failed to initialize. Will be ignored.", tok.c_str());
    }
  }
  return 0;
}

// topo.cc:1219-1284 — <msccl_algos><load path minbytes maxbytes proto/></msccl_algos>
int loadAlgosFromConfig(const char* path, std::vector<Algorithm>* algos, std::vector<Registration>* regs,
                        int maxNChannels, int rank, int nRanks) {
  INFO(kSubInit, "MSCCL: Parsing config %s", path);
  Loader L;
  MSCCLCHECK(readFile(path, &L.r.buf));
  MSCCLCHECK(L.loadSub(nullptr, kHMsccl));
  Node* top = L.findTag("msccl_algos");
  if (!top) { WARN("MSCCL: no <msccl_algos> in %s", path); return kInternal; }
  for (Node* n : top->subs) {
    if (n->name != "load") continue;
    if ((int)algos->size() == kMaxAlgos) {
      WARN("MSCCL: too many algorithms (%d) specified in environment variable MSCCL_XML_FILES. The rest will be ignored.", (int)algos->size());
      break;
    }
    const char* p;
    MSCCLCHECK(getAttrStr(n, "path", &p));
    int64_t minB = 0, maxB = -1;
    if (getAttr(n, "minbytes")) MSCCLCHECK(getAttrInt64(n, "minbytes", &minB));
    if (getAttr(n, "maxbytes")) MSCCLCHECK(getAttrInt64(n, "maxbytes", &maxB));
    const std::string* pr = getAttr(n, "proto");
    Algorithm a;
    if (loadAlgoFromXml(p, &a, maxNChannels, rank, nRanks) == 0) {
      Registration r;
      r.algoIndex = (int)algos->size();
      r.minBytes = minB;
      r.maxBytes = maxB;
      // A missing proto attribute makes the reference strcmp(NULL) (topo.cc:1276);
      // here it falls back to the protocol declared in the algorithm XML.
      if (pr) MSCCLCHECK(protoFromStr(pr->c_str(), &r.proto));
      else r.proto = a.proto;
      algos->push_back(std::move(a));
      regs->push_back(r);
      INFO(kSubInit, "Parsed MSCCL Algorithm %s successfully.", p);
    } else {
      WARN("MSCCL: algorithm %s failed to initialize. Will be ignored.", p);
    }
  }
  return 0;
}

std::string algoToJson(const Algorithm& a) {
  std::ostringstream o;
  o << "{\"name\":\"" << a.name << "\",\"valid\":" << (a.valid ? 1 : 0) << ",\"coll\":" << a.coll
    << ",\"inplace\":" << a.inPlace << ",\"ngpus\":" << a.ngpus << ",\"nchunksperloop\":" << a.nchunksPerLoop
    << ",\"proto\":" << a.proto << ",\"minBytes\":" << a.minBytes << ",\"maxBytes\":" << a.maxBytes
    << ",\"nchannels\":" << a.nChannels << ",\"nBlocks\":" << a.nBlocks << ",\"nthreads\":" << a.nThreads
    << ",\"nScratchChunks\":" << a.nScratchChunks << ",\"tbs\":[";
  for (int b = 0; b < (int)a.tbs.size(); b++) {
    const ThreadBlock& t = a.tbs[b];
    if (b) o << ",";
    o << "{\"send\":" << t.sendpeer << ",\"recv\":" << t.recvpeer << ",\"chan\":" << (int)t.channel
      << ",\"depBid\":[";
    for (size_t i = 0; i < t.depBid.size(); i++) o << (i ? "," : "") << t.depBid[i];
    o << "],\"depStep\":[";
    for (size_t i = 0; i < t.depStep.size(); i++) o << (i ? "," : "") << t.depStep[i];
    o << "],\"redSrcOff\":[";
    for (size_t i = 0; i < t.redSrcOff.size(); i++) o << (i ? "," : "") << t.redSrcOff[i];
    o << "],\"transfers\":[";
    for (size_t i = 0; i < t.transfers.size(); i++) {
      const Transfer& x = t.transfers[i];
      o << (i ? "," : "") << "[" << (int)x.type << "," << (int)x.srcbuf << "," << x.srcoff << ","
        << (int)x.dstbuf << "," << x.dstoff << "," << (int)x.count << "," << x.depPtr << "," << x.numDeps
        << "," << (int)x.hasDep << "," << x.redPtr << "," << x.numReds << "]";
    }
    o << "]}";
  }
  o << "]}";
  return o.str();
}

}  // namespace msccl
