"""Inert, byte-exact codec for scikit-learn-0.23.2 pickles (protocol 3).

The reference ships its fitted model only as ``hf_predict_model.pkl`` and reads it
with a bare ``pickle.load`` (reference ``predict_hf.py:33-34``).  That file was
written by scikit-learn 0.23.2 / numpy 1.x and can no longer be unpickled by a
modern scikit-learn (``sklearn.ensemble._gb_losses`` is gone and ``Tree`` rejects
the 7-field node dtype).  We therefore own the format:

* ``parse(bytes) -> Node``: an opcode-level reader that builds a graph of
  :class:`Node` records.  It never imports or calls anything named by the file
  (``GLOBAL`` becomes a :class:`Global` record), so it is safe on untrusted input.
* ``emit(Node) -> bytes``: a writer that re-serialises the graph following the
  exact opcode choices of CPython's protocol-3 ``_Pickler`` (memo order, batch
  sizes, TUPLE1/2/3, BININT1/2/BININT ...).  ``emit(parse(b)) == b`` for the
  shipped checkpoint (all 132,976 bytes; tested).
* ``to_py`` / ``Builder``: a value view (numpy arrays, :class:`SkObject`
  records) used by :mod:`hfens.io.checkpoint` to convert to and from the
  framework's native model objects.

Node identity is the memo: a node reachable twice is written once and then
referenced with ``BINGET``; two equal-valued but distinct nodes are written twice,
exactly as the original pickler did for distinct Python objects.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

__all__ = [
    "Node", "Prim", "Str", "Bytes", "TupleN", "ListN", "DictN", "Global", "Call",
    "parse", "emit", "to_py", "SkObject", "NpRandomState", "Builder",
]


# ----------------------------------------------------------------------------- nodes
class Node:
    __slots__ = ()


@dataclass(eq=False)
class Prim(Node):
    """int / float / bool / None (never memoised by the pickler)."""
    value: Any


@dataclass(eq=False)
class Str(Node):
    value: str


@dataclass(eq=False)
class Bytes(Node):
    value: bytes


@dataclass(eq=False)
class TupleN(Node):
    items: List[Node]


@dataclass(eq=False)
class ListN(Node):
    items: List[Node] = field(default_factory=list)


@dataclass(eq=False)
class DictN(Node):
    items: List[Tuple[Node, Node]] = field(default_factory=list)


@dataclass(eq=False)
class Global(Node):
    module: str
    name: str


@dataclass(eq=False)
class Call(Node):
    """Result of ``REDUCE`` (newobj=False) or ``NEWOBJ`` (newobj=True), plus any
    ``APPENDS``/``SETITEMS`` applied to it and an optional ``BUILD`` state."""
    func: Node
    args: Node
    newobj: bool
    listitems: List[Node] = field(default_factory=list)
    dictitems: List[Tuple[Node, Node]] = field(default_factory=list)
    state: Optional[Node] = None


# ----------------------------------------------------------------------------- reader
_MARK = object()


def parse(data: bytes) -> Node:
    """Decode a protocol<=3 pickle into a :class:`Node` graph without executing it."""
    stack: List[Any] = []
    memo: Dict[int, Node] = {}
    pos = 0
    n = len(data)

    def pop_mark() -> List[Any]:
        k = len(stack) - 1
        while stack[k] is not _MARK:
            k -= 1
        items = stack[k + 1:]
        del stack[k:]
        return items

    while pos < n:
        op = data[pos]
        pos += 1
        if op == 0x80:                      # PROTO
            if data[pos] > 3:
                raise ValueError(f"unsupported pickle protocol {data[pos]}")
            pos += 1
        elif op == 0x2E:                    # STOP
            if len(stack) != 1:
                raise ValueError("malformed pickle: stack depth %d at STOP" % len(stack))
            return stack[0]
        elif op == 0x63:                    # GLOBAL 'module\nname\n'
            e1 = data.index(b"\n", pos)
            e2 = data.index(b"\n", e1 + 1)
            stack.append(Global(data[pos:e1].decode("ascii"), data[e1 + 1:e2].decode("ascii")))
            pos = e2 + 1
        elif op == 0x71:                    # BINPUT
            memo[data[pos]] = stack[-1]
            pos += 1
        elif op == 0x72:                    # LONG_BINPUT
            memo[struct.unpack_from("<I", data, pos)[0]] = stack[-1]
            pos += 4
        elif op == 0x68:                    # BINGET
            stack.append(memo[data[pos]])
            pos += 1
        elif op == 0x6A:                    # LONG_BINGET
            stack.append(memo[struct.unpack_from("<I", data, pos)[0]])
            pos += 4
        elif op == 0x28:                    # MARK
            stack.append(_MARK)
        elif op == 0x29:                    # EMPTY_TUPLE
            stack.append(TupleN([]))
        elif op == 0x85:                    # TUPLE1
            stack[-1:] = [TupleN(stack[-1:])]
        elif op == 0x86:                    # TUPLE2
            stack[-2:] = [TupleN(stack[-2:])]
        elif op == 0x87:                    # TUPLE3
            stack[-3:] = [TupleN(stack[-3:])]
        elif op == 0x74:                    # TUPLE
            stack.append(TupleN(pop_mark()))
        elif op == 0x5D:                    # EMPTY_LIST
            stack.append(ListN())
        elif op == 0x7D:                    # EMPTY_DICT
            stack.append(DictN())
        elif op == 0x61:                    # APPEND
            v = stack.pop()
            _append(stack[-1], [v])
        elif op == 0x65:                    # APPENDS
            items = pop_mark()
            _append(stack[-1], items)
        elif op == 0x73:                    # SETITEM
            v = stack.pop()
            k = stack.pop()
            _setitems(stack[-1], [(k, v)])
        elif op == 0x75:                    # SETITEMS
            items = pop_mark()
            _setitems(stack[-1], list(zip(items[0::2], items[1::2])))
        elif op == 0x81:                    # NEWOBJ
            args = stack.pop()
            cls = stack.pop()
            stack.append(Call(cls, args, newobj=True))
        elif op == 0x52:                    # REDUCE
            args = stack.pop()
            func = stack.pop()
            stack.append(Call(func, args, newobj=False))
        elif op == 0x62:                    # BUILD
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, Call) or obj.state is not None:
                raise ValueError("BUILD on a non-object node")
            obj.state = state
        elif op == 0x58:                    # BINUNICODE
            ln = struct.unpack_from("<I", data, pos)[0]
            pos += 4
            stack.append(Str(data[pos:pos + ln].decode("utf-8", "surrogatepass")))
            pos += ln
        elif op == 0x43:                    # SHORT_BINBYTES
            ln = data[pos]
            pos += 1
            stack.append(Bytes(bytes(data[pos:pos + ln])))
            pos += ln
        elif op == 0x42:                    # BINBYTES
            ln = struct.unpack_from("<I", data, pos)[0]
            pos += 4
            stack.append(Bytes(bytes(data[pos:pos + ln])))
            pos += ln
        elif op == 0x4B:                    # BININT1
            stack.append(Prim(data[pos]))
            pos += 1
        elif op == 0x4D:                    # BININT2
            stack.append(Prim(struct.unpack_from("<H", data, pos)[0]))
            pos += 2
        elif op == 0x4A:                    # BININT
            stack.append(Prim(struct.unpack_from("<i", data, pos)[0]))
            pos += 4
        elif op == 0x8A:                    # LONG1
            ln = data[pos]
            pos += 1
            stack.append(Prim(int.from_bytes(data[pos:pos + ln], "little", signed=True)))
            pos += ln
        elif op == 0x47:                    # BINFLOAT
            stack.append(Prim(struct.unpack_from(">d", data, pos)[0]))
            pos += 8
        elif op == 0x4E:                    # NONE
            stack.append(Prim(None))
        elif op == 0x88:                    # NEWTRUE
            stack.append(Prim(True))
        elif op == 0x89:                    # NEWFALSE
            stack.append(Prim(False))
        else:
            raise ValueError(f"unsupported pickle opcode 0x{op:02x} at offset {pos - 1}")
    raise ValueError("pickle ended without STOP")


def _append(target, items):
    if isinstance(target, ListN):
        target.items.extend(items)
    elif isinstance(target, Call):
        target.listitems.extend(items)
    else:
        raise ValueError("APPEND(S) on a non-list node")


def _setitems(target, pairs):
    if isinstance(target, DictN):
        target.items.extend(pairs)
    elif isinstance(target, Call):
        target.dictitems.extend(pairs)
    else:
        raise ValueError("SETITEM(S) on a non-dict node")


# ----------------------------------------------------------------------------- writer
_BATCH = 1000  # pickle._Pickler._BATCHSIZE


class _Writer:
    def __init__(self):
        self.out = bytearray()
        self.memo: Dict[int, int] = {}

    # memo helpers ---------------------------------------------------------
    def _put(self, node: Node):
        idx = len(self.memo)
        self.memo[id(node)] = idx
        if idx < 256:
            self.out += b"q" + bytes([idx])
        else:
            self.out += b"r" + struct.pack("<I", idx)

    def _get(self, idx: int):
        if idx < 256:
            self.out += b"h" + bytes([idx])
        else:
            self.out += b"j" + struct.pack("<I", idx)

    # ---------------------------------------------------------------------
    def save(self, node: Node):
        if isinstance(node, Prim):
            self._prim(node.value)
            return
        if isinstance(node, TupleN) and not node.items:
            self.out += b")"
            return
        got = self.memo.get(id(node))
        if got is not None:
            self._get(got)
            return
        if isinstance(node, Str):
            raw = node.value.encode("utf-8", "surrogatepass")
            self.out += b"X" + struct.pack("<I", len(raw)) + raw
            self._put(node)
        elif isinstance(node, Bytes):
            v = node.value
            if len(v) < 256:
                self.out += b"C" + bytes([len(v)]) + v
            else:
                self.out += b"B" + struct.pack("<I", len(v)) + v
            self._put(node)
        elif isinstance(node, Global):
            self.out += b"c" + node.module.encode("ascii") + b"\n" + node.name.encode("ascii") + b"\n"
            self._put(node)
        elif isinstance(node, TupleN):
            k = len(node.items)
            if k <= 3:
                for it in node.items:
                    self.save(it)
                self.out += (b"\x85", b"\x86", b"\x87")[k - 1]
            else:
                self.out += b"("
                for it in node.items:
                    self.save(it)
                self.out += b"t"
            self._put(node)
        elif isinstance(node, ListN):
            self.out += b"]"
            self._put(node)
            self._appends(node.items)
        elif isinstance(node, DictN):
            self.out += b"}"
            self._put(node)
            self._setitems(node.items)
        elif isinstance(node, Call):
            self.save(node.func)
            self.save(node.args)
            self.out += b"\x81" if node.newobj else b"R"
            self._put(node)
            if node.listitems:
                self._appends(node.listitems)
            if node.dictitems:
                self._setitems(node.dictitems)
            if node.state is not None:
                self.save(node.state)
                self.out += b"b"
        else:
            raise TypeError(f"cannot emit {type(node).__name__}")

    def _prim(self, v):
        if v is None:
            self.out += b"N"
        elif v is True:
            self.out += b"\x88"
        elif v is False:
            self.out += b"\x89"
        elif isinstance(v, int):
            if 0 <= v < 0x100:
                self.out += b"K" + bytes([v])
            elif 0 <= v < 0x10000:
                self.out += b"M" + struct.pack("<H", v)
            elif -0x80000000 <= v <= 0x7FFFFFFF:
                self.out += b"J" + struct.pack("<i", v)
            else:
                raw = v.to_bytes((v.bit_length() + 8) // 8, "little", signed=True)
                self.out += b"\x8a" + bytes([len(raw)]) + raw
        elif isinstance(v, float):
            self.out += b"G" + struct.pack(">d", v)
        else:
            raise TypeError(f"unsupported primitive {type(v)}")

    def _appends(self, items):
        for i in range(0, len(items), _BATCH):
            batch = items[i:i + _BATCH]
            if len(batch) > 1:
                self.out += b"("
                for it in batch:
                    self.save(it)
                self.out += b"e"
            else:
                self.save(batch[0])
                self.out += b"a"

    def _setitems(self, pairs):
        for i in range(0, len(pairs), _BATCH):
            batch = pairs[i:i + _BATCH]
            if len(batch) > 1:
                self.out += b"("
                for k, v in batch:
                    self.save(k)
                    self.save(v)
                self.out += b"u"
            else:
                k, v = batch[0]
                self.save(k)
                self.save(v)
                self.out += b"s"


def emit(root: Node) -> bytes:
    """Serialise a node graph exactly as CPython's protocol-3 pickler would."""
    w = _Writer()
    w.out += b"\x80\x03"
    w.save(root)
    w.out += b"."
    return bytes(w.out)


# ----------------------------------------------------------------------------- value view
@dataclass
class SkObject:
    """An estimator-like record: ``cls`` = 'module.Name', ordered ``state`` dict,
    optional constructor ``args`` (REDUCE objects such as ``Tree``) and ``items``
    (dict-subclass payload such as ``Bunch``)."""
    cls: str
    state: Any = None
    args: tuple = ()
    items: Optional[dict] = None

    def __getitem__(self, k):
        return self.state[k]


@dataclass
class NpRandomState:
    """numpy ``RandomState`` pickled via ``__randomstate_ctor`` (MT19937)."""
    key: np.ndarray
    pos: int
    has_gauss: int = 0
    gauss: float = 0.0
    bit_generator: str = "MT19937"


_RECON = ("numpy.core.multiarray", "_reconstruct")
_SCALAR = ("numpy.core.multiarray", "scalar")
_DTYPE = ("numpy", "dtype")
_RSCTOR = ("numpy.random._pickle", "__randomstate_ctor")


def _gname(n: Node) -> Tuple[str, str]:
    return (n.module, n.name) if isinstance(n, Global) else ("", "")


def _dtype_from(node: Call) -> np.dtype:
    args = to_py(node.args)
    st = to_py(node.state) if node.state is not None else None
    base = args[0]
    if st is None:
        return np.dtype(base)
    # state = (version, byteorder, subdescr, names, fields, elsize, alignment, flags)
    ver, order = st[0], st[1]
    names, fields = st[3], st[4]
    if names is None:
        dt = np.dtype(base)
        if order in ("<", ">") and dt.itemsize > 1:
            dt = dt.newbyteorder(order)
        return dt
    spec = {"names": [], "formats": [], "offsets": []}
    for nm in names:
        sub, off = fields[nm][0], fields[nm][1]
        spec["names"].append(nm)
        spec["formats"].append(sub)
        spec["offsets"].append(off)
    spec["itemsize"] = st[5]
    return np.dtype(spec)


def to_py(node: Node, _cache: Optional[dict] = None) -> Any:
    """Value view of a node graph (numpy arrays, SkObject records).  Shared
    nodes map to shared Python objects."""
    if _cache is None:
        _cache = {}
    key = id(node)
    if key in _cache:
        return _cache[key]
    if isinstance(node, Prim):
        return node.value
    if isinstance(node, (Str, Bytes)):
        return node.value
    if isinstance(node, Global):
        v = f"{node.module}.{node.name}"
    elif isinstance(node, TupleN):
        v = tuple(to_py(i, _cache) for i in node.items)
    elif isinstance(node, ListN):
        v = []
        _cache[key] = v
        v.extend(to_py(i, _cache) for i in node.items)
        return v
    elif isinstance(node, DictN):
        v = {}
        _cache[key] = v
        for k, x in node.items:
            v[to_py(k, _cache)] = to_py(x, _cache)
        return v
    elif isinstance(node, Call):
        g = _gname(node.func)
        if g == _RECON:
            ver, shape, dt, fortran, raw = node.state.items
            dtype = _dtype_from(dt) if isinstance(dt, Call) else np.dtype(to_py(dt, _cache))
            shape = to_py(shape, _cache)
            if dtype.hasobject:
                flat = np.empty(int(np.prod(shape)), dtype=object)
                flat[:] = to_py(raw, _cache)
                v = flat.reshape(shape, order="F" if to_py(fortran) else "C")
            else:
                v = np.frombuffer(to_py(raw, _cache), dtype=dtype).reshape(
                    shape, order="F" if to_py(fortran) else "C").copy()
        elif g == _DTYPE:
            v = _dtype_from(node)
        elif g == _SCALAR:
            dt, raw = node.args.items
            dtype = _dtype_from(dt)
            v = np.frombuffer(to_py(raw, _cache), dtype=dtype)[0]
        elif g == _RSCTOR:
            st = to_py(node.state, _cache)
            v = NpRandomState(key=st["state"]["key"], pos=st["state"]["pos"],
                              has_gauss=st["has_gauss"], gauss=st["gauss"],
                              bit_generator=st["bit_generator"])
        else:
            cls = "%s.%s" % g
            v = SkObject(cls=cls, args=to_py(node.args, _cache))
            _cache[key] = v
            v.state = to_py(node.state, _cache) if node.state is not None else None
            if node.dictitems:
                v.items = {to_py(k, _cache): to_py(x, _cache) for k, x in node.dictitems}
            return v
    else:
        raise TypeError(type(node))
    _cache[key] = v
    return v


# ----------------------------------------------------------------------------- builder
class Builder:
    """Build node graphs for *fresh* checkpoints with the same sharing conventions
    numpy-1.x / sklearn-0.23.2 produced: one ``GLOBAL`` node per class path, the
    ``ndarray``/``b'b'`` reconstruct constants and dtype objects shared across
    arrays, attribute-name strings interned (shared) per object graph."""

    def __init__(self):
        self._globals: Dict[Tuple[str, str], Global] = {}
        self._interned: Dict[str, Str] = {}
        self._dtypes: Dict[str, Call] = {}
        self._bb = Bytes(b"b")

    def g(self, module: str, name: str) -> Global:
        k = (module, name)
        if k not in self._globals:
            self._globals[k] = Global(module, name)
        return self._globals[k]

    def s(self, text: str) -> Str:
        """Interned string (identifiers, constants: shared by the pickler's memo)."""
        if text not in self._interned:
            self._interned[text] = Str(text)
        return self._interned[text]

    @staticmethod
    def fresh(text: str) -> Str:
        """A runtime-created string (not shared)."""
        return Str(text)

    def prim(self, v) -> Prim:
        return Prim(v)

    def dtype(self, dt: np.dtype) -> Call:
        dt = np.dtype(dt)
        key = dt.str if dt.names is None else repr(dt.descr)
        if key in self._dtypes:
            return self._dtypes[key]
        if dt.names is None:
            code = {"f": "f", "i": "i", "u": "u", "b": "b", "O": "O"}[dt.kind] + str(dt.itemsize)
            if dt.kind == "O":
                code = "O8"
            if dt.kind == "b":
                code = "b1"
            order = "|" if dt.itemsize == 1 or dt.kind == "O" else "<"
            st = TupleN([Prim(3), self.s(order), Prim(None), Prim(None), Prim(None),
                         Prim(-1), Prim(-1), Prim(63 if dt.kind == "O" else 0)])
            node = Call(self.g(*_DTYPE), TupleN([self.s(code), Prim(False), Prim(True)]),
                        newobj=False, state=st)
        else:
            names = TupleN([self.s(n) for n in dt.names])
            fields = DictN([(self.s(n), TupleN([self.dtype(dt.fields[n][0]), Prim(dt.fields[n][1])]))
                            for n in dt.names])
            st = TupleN([Prim(3), self.s("|"), Prim(None), names, fields,
                         Prim(dt.itemsize), Prim(1), Prim(16)])
            node = Call(self.g(*_DTYPE), TupleN([self.s("V%d" % dt.itemsize), Prim(False), Prim(True)]),
                        newobj=False, state=st)
        self._dtypes[key] = node
        return node

    def array(self, a: np.ndarray, obj_items: Optional[List[Node]] = None) -> Call:
        a = np.asarray(a)
        shape = TupleN([Prim(int(d)) for d in a.shape])
        if a.dtype.hasobject:
            raw = ListN(list(obj_items))
        else:
            raw = Bytes(np.ascontiguousarray(a).tobytes())
        state = TupleN([Prim(1), shape, self.dtype(a.dtype), Prim(False), raw])
        return Call(self.g(*_RECON), TupleN([self.g("numpy", "ndarray"), TupleN([Prim(0)]), self._bb]),
                    newobj=False, state=state)

    def scalar(self, x: np.generic) -> Call:
        x = np.asarray(x)
        return Call(self.g(*_SCALAR), TupleN([self.dtype(x.dtype), Bytes(x.tobytes())]), newobj=False)

    def obj(self, module: str, name: str, state: List[Tuple[str, Node]]) -> Call:
        st = DictN([(self.s(k), v) for k, v in state])
        return Call(self.g(module, name), TupleN([]), newobj=True, state=st)

    def randomstate(self, rs: NpRandomState) -> Call:
        mt = self.s("MT19937")
        inner = DictN([(self.s("key"), self.array(np.asarray(rs.key, dtype=np.uint32))),
                       (self.s("pos"), Prim(int(rs.pos)))])
        st = DictN([(self.s("bit_generator"), mt), (self.s("state"), inner),
                    (self.s("has_gauss"), Prim(int(rs.has_gauss))), (self.s("gauss"), Prim(float(rs.gauss)))])
        return Call(self.g(*_RSCTOR), TupleN([mt]), newobj=False, state=st)

    def value(self, v) -> Node:
        """Generic Python value → node (ints, floats, strings, tuples, lists, arrays)."""
        if isinstance(v, Node):
            return v
        if v is None or isinstance(v, (bool, int, float)) and not isinstance(v, np.generic):
            return Prim(v)
        if isinstance(v, str):
            return self.s(v)
        if isinstance(v, np.ndarray):
            return self.array(v)
        if isinstance(v, np.generic):
            return self.scalar(v)
        if isinstance(v, tuple):
            return TupleN([self.value(x) for x in v])
        if isinstance(v, list):
            return ListN([self.value(x) for x in v])
        raise TypeError(type(v))
