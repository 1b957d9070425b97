"""ORACLE (test infrastructure only) — CPU restatement of the reference's MSCCL XML loader.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker.  The product loader is msccl_amd/csrc/xml.cc.

Restates (behaviour, not code):
  * tokenizer            /root/reference/src/graph/xml.cc:20-211
      - whitespace between elements is only ' ', '\\n', '\\r' (xml.cc:109)
      - attribute values open with ' or " but always close at '"' (xml.cc:28-55)
      - names end at ' ', '>', '/', '\\n', '\\r' (xml.cc:57-80), max 255 chars
      - <!-- comments --> (xml.cc:84-104)
      - more than 16 attributes: the extras are parsed and dropped (xml.cc:136-140)
      - unknown elements are skipped; inside a skipped element any closing tag ends
        the level (the child is parsed into the parent's node slot, xml.cc:170-208)
      - at most 4096 retained nodes (xml.h:19, xml.cc:171-174)
  * rank filtering       xml.cc:850-893  (only <gpu id==rank> children are retained)
  * integer attributes   xml.h:105-117   (strtol(str, NULL, 0): base prefix, stops at junk)
  * algorithm building   graph/topo.cc:759-1193
  * file list            graph/topo.cc:1195-1217  (MSCCL_XML_FILES)

Parity pin: the resulting program is compared (tests/test_oracle_loader.py) with the
reference loader's own output on the RCCL-shipped msccl-tools XMLs as recorded by the
survey session that compiled the reference loader, and with the
product loader on every fixture.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

# limits (include/msccl.h:6-14, devcomm.h:33)
MAX_STEPS = 256
MAX_TB = 216
MAX_COUNT = 72
MAX_REDUCE_FUSION = 16
MAXCHANNELS = 32
MAX_ALGOS = 4
MAX_STR_LEN = 255
MAX_ATTR_COUNT = 16
MAX_SUBS = 1024
MAX_NODES = 1 << 12

# ncclResult_t
SUCCESS, SYSTEM, INTERNAL, INVALID_USAGE = 0, 2, 3, 5

# buffers (msccl.h:19-21) / transfer types (msccl.h:23-31)
INPUT, OUTPUT, SCRATCH = 0, 1, 2
SEND, RECV, RCS, RRS, RRC, RRCS, CPY, RE, RA = range(9)
TYPE_NAMES = {"s": SEND, "r": RECV, "rcs": RCS, "rrs": RRS, "rrc": RRC, "rrcs": RRCS,
              "cpy": CPY, "re": RE, "ra": RA, "nop": -1}
PROTO_LL, PROTO_LL128, PROTO_SIMPLE = 0, 1, 2
# ncclFunc_t (devcomm.h:16)
BROADCAST, REDUCE_COLL, ALLGATHER, REDUCE_SCATTER, ALLREDUCE, ALLTOALL, CUSTOM = range(7)

NONE_T, OPEN_T, CLOSE_T, SINGLE_T = 0, 1, 2, 3


class XmlError(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


@dataclasses.dataclass
class Node:
    name: str = ""
    attrs: List[Tuple[str, str]] = dataclasses.field(default_factory=list)
    type: int = NONE_T
    subs: List["Node"] = dataclasses.field(default_factory=list)

    def attr(self, key: str) -> Optional[str]:
        for k, v in self.attrs:
            if k == key:
                return v
        return None


class _Reader:
    def __init__(self, data: str):
        self.data = data
        self.pos = 0

    def get(self) -> Optional[str]:
        if self.pos >= len(self.data):
            return None
        c = self.data[self.pos]
        self.pos += 1
        return c

    def need(self) -> str:
        c = self.get()
        if c is None:
            raise XmlError(INTERNAL, "XML Parse : Unexpected EOF")
        return c


def _get_value(r: _Reader) -> Tuple[str, str]:
    c = r.need()
    if c not in ('"', "'"):
        raise XmlError(INTERNAL, "XML Parse : Expected (double) quote.")
    out = []
    while True:
        c = r.need()
        if c == '"':
            break
        out.append(c)
        if len(out) > MAX_STR_LEN:
            raise XmlError(INTERNAL, "value too long")
    return "".join(out), r.need()


def _get_token(r: _Reader, want_value: bool):
    name = []
    while True:
        c = r.need()
        if c == "=":
            if not want_value:
                raise XmlError(INTERNAL, "XML Parse : Unexpected value with name %s" % "".join(name))
            v, last = _get_value(r)
            return "".join(name), v, last
        name.append(c)
        if len(name) == MAX_STR_LEN:
            raise XmlError(INTERNAL, "name too long")
        if c in (" ", ">", "/", "\n", "\r"):
            break
    return "".join(name[:-1]), None, name[-1]


def _skip_comment(r: _Reader, start: str, nxt: str) -> None:
    end = "..."
    for ch in start + nxt:
        end = end[1:] + ch
    while end != "-->":
        c = r.get()
        if c is None:
            raise XmlError(INTERNAL, "XML Parse error : unterminated comment")
        end = end[1:] + c


def _get_node(r: _Reader) -> Node:
    node = Node()
    c = " "
    while c in (" ", "\n", "\r"):
        c = r.get()
        if c is None:
            return node  # NONE
    if c != "<":
        raise XmlError(INTERNAL, "XML Parse error : expecting '<', got %r" % c)
    name, _, c = _get_token(r, False)
    if name.startswith("!--"):
        _skip_comment(r, name[3:], c)
        return _get_node(r)
    if name == "" and c == "/":
        name, _, c = _get_token(r, False)
        if c != ">":
            raise XmlError(INTERNAL, "unexpected trailing %r in closing tag %s" % (c, name))
        return Node(name=name, type=CLOSE_T)
    node.name = name
    node.type = OPEN_T
    while c == " ":
        k, v, c = _get_token(r, True)
        if len(node.attrs) < MAX_ATTR_COUNT:
            node.attrs.append((k, v if v is not None else ""))
    if c == "/":
        node.type = SINGLE_T
        _, _, c = _get_token(r, False)
    if c != ">":
        raise XmlError(INTERNAL, "XML Parse : expected >, got %r" % c)
    return node


class _Doc:
    def __init__(self, data: str, myrank: int):
        self.r = _Reader(data)
        self.nodes: List[Node] = []
        self.myrank = myrank

    def skip(self, head_type: int) -> None:
        if head_type == SINGLE_T:
            return
        while True:
            n = _get_node(self.r)
            if n.type == NONE_T:
                raise XmlError(INTERNAL, "XML Parse : unterminated element")
            if n.type == CLOSE_T:
                return
            self.skip(n.type)

    def load_sub(self, head: Optional[Node], handler: Optional[str]) -> None:
        if head is not None and head.type == SINGLE_T:
            return
        while True:
            if len(self.nodes) == MAX_NODES:
                raise XmlError(INTERNAL, "Error : XML parser is limited to %d nodes" % MAX_NODES)
            n = _get_node(self.r)
            if n.type == NONE_T:
                if head is not None:
                    raise XmlError(INTERNAL, "XML Parse : unterminated %s" % head.name)
                return
            if head is not None and n.type == CLOSE_T:
                if n.name != head.name:
                    raise XmlError(INTERNAL, "XML Mismatch : %s / %s" % (head.name, n.name))
                return
            if handler is not None and n.name == handler:
                if head is not None:
                    if len(head.subs) == MAX_SUBS:
                        raise XmlError(INTERNAL, "too many children")
                    head.subs.append(n)
                self.nodes.append(n)
                self.handle(handler, n)
            else:
                self.skip(n.type)

    def handle(self, handler: str, n: Node) -> None:
        if handler == "algo":
            self.load_sub(n, "gpu")
        elif handler == "gpu":
            if _strtol(_attr_str(n, "id")) == self.myrank:
                self.load_sub(n, "tb")
            else:
                self.load_sub(n, None)
        elif handler == "tb":
            self.load_sub(n, "step")
        elif handler == "step":
            if n.type != SINGLE_T:
                raise XmlError(INTERNAL, "<step> must be self-closing")
        elif handler == "msccl_algos":
            self.load_sub(n, "load")
        elif handler == "load":
            self.load_sub(n, None)


def _strtol(s: str) -> int:
    """C strtol(s, NULL, 0): optional space/sign, 0x hex, leading-0 octal, stop at junk."""
    i, n = 0, len(s)
    while i < n and s[i] in " \t\n\r\f\v":
        i += 1
    neg = False
    if i < n and s[i] in "+-":
        neg = s[i] == "-"
        i += 1
    base = 10
    if i + 1 < n and s[i] == "0" and s[i + 1] in "xX" and i + 2 < n and s[i + 2] in "0123456789abcdefABCDEF":
        base, i = 16, i + 2
    elif i < n and s[i] == "0":
        base = 8
    digits = "0123456789abcdef"[:base]
    v = 0
    while i < n and s[i].lower() in digits:
        v = v * base + digits.index(s[i].lower())
        i += 1
    return -v if neg else v


def _c_int(v: int) -> int:
    """truncate a C long to int, as `*value = strtol(...)` into an int does."""
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def _attr_str(n: Node, key: str) -> str:
    v = n.attr(key)
    if v is None:
        raise XmlError(INTERNAL, "Attribute %s of node %s not found" % (key, n.name))
    return v


def _attr_int(n: Node, key: str) -> int:
    return _c_int(_strtol(_attr_str(n, key)))


def _attr_int64(n: Node, key: str) -> int:
    return _strtol(_attr_str(n, key))


@dataclasses.dataclass
class Transfer:
    type: int
    srcbuf: int
    srcoff: int
    dstbuf: int
    dstoff: int
    count: int
    depPtr: int = 0
    numDeps: int = 0
    hasDep: int = 0
    redPtr: int = 0
    numReds: int = 0

    def as_list(self):
        return [self.type, self.srcbuf, self.srcoff, self.dstbuf, self.dstoff, self.count,
                self.depPtr, self.numDeps, self.hasDep, self.redPtr, self.numReds]


@dataclasses.dataclass
class ThreadBlock:
    send: int = -1
    recv: int = -1
    chan: int = 0
    depBid: List[int] = dataclasses.field(default_factory=list)
    depStep: List[int] = dataclasses.field(default_factory=list)
    redSrcOff: List[int] = dataclasses.field(default_factory=list)
    transfers: List[Transfer] = dataclasses.field(default_factory=list)


@dataclasses.dataclass
class Algorithm:
    name: str = ""
    valid: bool = False
    coll: int = ALLREDUCE
    inplace: int = 0
    ngpus: int = 0
    nchunksperloop: int = 0
    proto: int = PROTO_SIMPLE
    minBytes: int = 0
    maxBytes: int = 1 << 27
    nchannels: int = 0
    nBlocks: int = 0
    nthreads: int = 0
    nScratchChunks: int = 0
    nInputChunks: int = 0
    nOutputChunks: int = 0
    tbs: List[ThreadBlock] = dataclasses.field(default_factory=list)

    def to_dict(self) -> Dict:
        return {
            "name": self.name, "valid": int(self.valid), "coll": self.coll, "inplace": self.inplace,
            "ngpus": self.ngpus, "nchunksperloop": self.nchunksperloop, "proto": self.proto,
            "minBytes": self.minBytes, "maxBytes": self.maxBytes, "nchannels": self.nchannels,
            "nBlocks": self.nBlocks, "nthreads": self.nthreads, "nScratchChunks": self.nScratchChunks,
            "tbs": [{"send": t.send, "recv": t.recv, "chan": t.chan, "depBid": list(t.depBid),
                     "depStep": list(t.depStep), "redSrcOff": list(t.redSrcOff),
                     "transfers": [x.as_list() for x in t.transfers]} for t in self.tbs],
        }


def _proto_id(p: str) -> int:
    # topo.cc:745-757
    if p == "Simple":
        return PROTO_SIMPLE
    if p == "LL128":
        return PROTO_LL128
    if p == "LL":
        return PROTO_LL
    raise XmlError(INVALID_USAGE, "MSCCL: protocol %s is not supported." % p)


def _buffer_type(s: str) -> int:
    # topo.cc:711-723
    m = {"i": INPUT, "o": OUTPUT, "s": SCRATCH}
    if s not in m:
        raise XmlError(INVALID_USAGE, "type of buffer is not supported: %s" % s)
    return m[s]


def _check_bounds(buf: int, off: int, nin: int, nout: int, nscr: int) -> None:
    # topo.cc:725-743
    lim = {INPUT: nin, OUTPUT: nout, SCRATCH: nscr}[buf]
    if off < -1 or off >= lim:
        raise XmlError(INVALID_USAGE, "Incorrect offset %d for buffer %d (max %d)" % (off, buf, lim))


def parse_xml(data: str, rank: int, nranks: int, max_nchannels: int = MAXCHANNELS) -> Algorithm:
    """topo.cc:759-1193 on the text of one XML file.  Raises XmlError on rejection."""
    doc = _Doc(data, rank)
    doc.load_sub(None, "algo")
    top = next((n for n in doc.nodes if n.name == "algo"), None)
    if top is None:
        raise XmlError(INTERNAL, "no <algo> element")
    a = Algorithm()
    a.name = _attr_str(top, "name")[:63]
    ngpus = _attr_int(top, "ngpus")
    if ngpus != nranks:
        raise XmlError(INVALID_USAGE, "MSCCL: ngpus (%d) != nRanks (%d)" % (ngpus, nranks))
    a.ngpus = ngpus
    ncpl = _attr_int(top, "nchunksperloop")
    nch = _attr_int(top, "nchannels")
    a.proto = _proto_id(_attr_str(top, "proto"))
    min_b = _attr_int64(top, "minBytes") if top.attr("minBytes") is not None else 0
    max_b = _attr_int64(top, "maxBytes") if top.attr("maxBytes") is not None else (1 << 27)
    if min_b > max_b:
        raise XmlError(INVALID_USAGE, "MSCCL: minBytes cannot be greater than maxBytes.")
    if min_b < 0:
        raise XmlError(INVALID_USAGE, "MSCCL: minBytes cannot be negative.")
    if max_b < 0:
        raise XmlError(INVALID_USAGE, "MSCCL: maxBytes cannot be negative.")
    a.minBytes, a.maxBytes = min_b, max_b
    coll = _attr_str(top, "coll")
    in_mul = out_mul = 1
    colls = {"allreduce": ALLREDUCE, "allgather": ALLGATHER, "reduce": REDUCE_COLL,
             "broadcast": BROADCAST, "alltoall": ALLTOALL, "reduce_scatter": REDUCE_SCATTER,
             "custom": CUSTOM}
    if coll not in colls:
        raise XmlError(INVALID_USAGE, "MSCCL: collective type %s is not supported." % coll)
    a.coll = colls[coll]
    if coll == "allgather":
        in_mul = nranks
    if coll == "reduce_scatter":
        out_mul = nranks
    a.inplace = 1 if _attr_int(top, "inplace") else 0
    if top.attr("nthreads") is not None:
        a.nthreads = _attr_int(top, "nthreads")
        if a.nthreads % 32 != 0:
            raise XmlError(INVALID_USAGE, "MSCCL nthreads must be a multiplication of 32")
    a.nchannels = nch
    a.nchunksperloop = ncpl

    tbs: Dict[int, ThreadBlock] = {}
    exists = [False] * MAX_TB
    for g in top.subs:
        if g.name != "gpu":
            continue
        gid = _attr_int(g, "id")
        if gid != rank:
            continue
        nin = _attr_int(g, "i_chunks")
        nout = _attr_int(g, "o_chunks")
        nscr = _attr_int(g, "s_chunks")
        if nscr < 0:
            raise XmlError(INVALID_USAGE, "MSCCL: nScratchChunks must be not negative")
        if (nin > 0 and nin * in_mul != ncpl) or (nout > 0 and nout * out_mul != ncpl):
            raise XmlError(INVALID_USAGE, "Inconsistency between i_chunks/o_chunks and nchunksperloop")
        a.nScratchChunks, a.nInputChunks, a.nOutputChunks = nscr, nin, nout
        for tbn in g.subs:
            if tbn.name != "tb":
                continue
            bid = _attr_int(tbn, "id")
            recvpeer = _attr_int(tbn, "recv")
            sendpeer = _attr_int(tbn, "send")
            chan = _attr_int(tbn, "chan")
            if bid < 0 or bid >= MAX_TB:
                raise XmlError(INVALID_USAGE, "bad tb id %d" % bid)
            if exists[bid]:
                raise XmlError(INVALID_USAGE, "MSCCL: duplicate thread block id %d" % bid)
            exists[bid] = True
            if recvpeer == gid or sendpeer == gid:
                raise XmlError(INVALID_USAGE, "peer and gpu id must be different")
            if recvpeer < -1 or sendpeer < -1 or recvpeer >= ngpus or sendpeer >= ngpus:
                raise XmlError(INVALID_USAGE, "bad peer")
            if chan < 0 or chan >= MAXCHANNELS:
                raise XmlError(INVALID_USAGE, "invalid channel %d" % chan)
            tb = ThreadBlock(send=sendpeer, recv=recvpeer, chan=chan)
            old_dep_ptr = 0
            old_dst_buf = old_dst_off = old_src_buf = -1
            for st in tbn.subs:
                if st.name != "step":
                    continue
                s = _attr_int(st, "s")
                srcoff = _attr_int(st, "srcoff")
                srcbuf = _attr_str(st, "srcbuf")
                dstoff = _attr_int(st, "dstoff")
                dstbuf = _attr_str(st, "dstbuf")
                count = _attr_int(st, "cnt")
                typ = _attr_str(st, "type")
                dep_bid = _attr_int(st, "depid")
                dep_step = _attr_int(st, "deps")
                has_dep = _attr_int(st, "hasdep")
                if s >= MAX_STEPS:
                    raise XmlError(INTERNAL, "MSCCL: too many steps are requested")
                if s < 0:
                    raise XmlError(INTERNAL, "MSCCL: step must be positive")
                if typ not in TYPE_NAMES:
                    raise XmlError(INTERNAL, "MSCCL: type of transfer is not supported: %s" % typ)
                tt = TYPE_NAMES[typ]
                has_send = tt in (SEND, RCS, RRS, RRCS)
                has_recv = tt in (RECV, RCS, RRS, RRC, RRCS)
                check_src = tt in (SEND, RRS, RRCS, CPY, RE, RA)
                check_dst = tt in (RECV, RCS, RRCS, CPY, RE, RA)
                if dep_bid >= 0:
                    tb.depBid.append(dep_bid)
                    tb.depStep.append(dep_step)
                sb = _buffer_type(srcbuf)
                db = _buffer_type(dstbuf)
                continuation = False
                if tt == RE:
                    if old_dst_buf == db and old_dst_off == dstoff and old_src_buf == sb and dep_bid == -1:
                        continuation = True
                    else:
                        old_dst_buf = old_dst_off = -1
                if tt == -1:
                    continue
                if count < 0 or count >= MAX_COUNT:
                    raise XmlError(INTERNAL, "MSCCL: count (%d) out of range" % count)
                if has_send and sendpeer < 0:
                    raise XmlError(INVALID_USAGE, "send without sendpeer")
                if has_recv and recvpeer < 0:
                    raise XmlError(INVALID_USAGE, "recv without recvpeer")
                if check_src:
                    _check_bounds(sb, srcoff, nin, nout, nscr)
                if check_dst:
                    _check_bounds(db, dstoff, nin, nout, nscr)
                if continuation:
                    t = tb.transfers[-1]
                    t.type, t.srcbuf, t.srcoff, t.dstbuf, t.dstoff, t.count = tt, sb, srcoff, db, dstoff, count
                else:
                    if len(tb.transfers) >= MAX_STEPS:
                        raise XmlError(INVALID_USAGE, "too many steps")
                    t = Transfer(tt, sb, srcoff, db, dstoff, count)
                    t.depPtr = old_dep_ptr
                    t.numDeps = len(tb.depBid) - old_dep_ptr
                    if t.numDeps > 0 and dep_bid < 0:
                        raise XmlError(INVALID_USAGE, "dependence chain must end on a transfer with depid")
                    old_dep_ptr = len(tb.depBid)
                    tb.transfers.append(t)
                if tt != RE:
                    old_dst_buf = old_dst_off = old_src_buf = -1
                else:
                    if old_dst_buf == -1:
                        t.redPtr = len(tb.redSrcOff)
                    tb.redSrcOff.append(srcoff)
                    t.numReds = len(tb.redSrcOff) - t.redPtr
                    if has_dep or len(tb.redSrcOff) == MAX_REDUCE_FUSION:
                        old_dst_buf = old_dst_off = -1
                    else:
                        old_dst_buf, old_dst_off, old_src_buf = db, dstoff, sb
                    if t.numReds > MAX_REDUCE_FUSION:
                        raise XmlError(INVALID_USAGE, "reduction chain too long")
                if has_dep not in (0, 1):
                    raise XmlError(INTERNAL, "has_dependence must be 0 or 1")
                t.hasDep = has_dep
            tbs[bid] = tb
        nb = 1 if exists[0] else 0
        for i in range(1, MAX_TB):
            if exists[i] and not exists[i - 1]:
                raise XmlError(INVALID_USAGE, "MSCCL: threadblock %d is missing" % i)
            if exists[i]:
                nb = i + 1
        a.nBlocks = nb
    a.tbs = [tbs[i] for i in range(a.nBlocks)]
    a.valid = True
    return a


def load_xml(path: str, rank: int, nranks: int, max_nchannels: int = MAXCHANNELS) -> Algorithm:
    with open(path, "r", encoding="latin-1") as f:
        return parse_xml(f.read(), rank, nranks, max_nchannels)


def load_xml_files(paths: str, rank: int, nranks: int) -> List[Algorithm]:
    """topo.cc:1195-1217: ':'-separated list, failed files skipped, at most 4 loaded."""
    out = []
    for tok in [t for t in paths.split(":") if t]:
        if len(out) == MAX_ALGOS:
            break
        try:
            out.append(load_xml(tok, rank, nranks))
        except (XmlError, OSError):
            pass
    return out
