"""Restatement of the Java Object Serialization stream (java.io.ObjectOutputStream,
protocol version 2) for the one object IPLS serialises on the aggregation path:
the partial update ``new org.javatuples.Pair<>(workers, gradients)`` with
``Integer workers`` and ``double[] gradients``.

TEST INFRASTRUCTURE ONLY: the checker of ``ipls_pair_parse`` /
``ipls_pair_encode`` / ``IPLS_HOST_PAIR`` (include/ipls_agg.h).  Nothing in the
product imports this module.

Where the reference writes and reads it:
  * MyIPFSClass.Update_file(String, Pair<Integer,double[]>)   MyIPFSClass.java:160-166
    (ObjectOutputStream.writeObject of the Pair) -- called by
    IPLS_Comm.commit_partial_update (IPLS_Comm.java:56-58, local_save) and by
    DStorage_Client.sendPartition(..., double[] data, mod == 1)
    (DStorage_Client.java:152-154, -i 1 indirect communication, from
    IPLS.java:1423-1425);
  * MyIPFSClass.Download_Partial_Updates(hash)                MyIPFSClass.java:326-338
    (ObjectInputStream.readObject) -- read by Download_Scheduler
    (:324-325, the replica partial folded into REP) and by the storage node's
    merge when status != 0 (Decentralized_Storage_Receiver.java:249-256).

The byte layout follows the serialization grammar (stream magic, TC_* tags,
class descriptors with their serialVersionUIDs, handles from 0x7e0000).  The
descriptor bytes are pinned by data the reference itself wrote: its
``Scheduler`` file (an ObjectOutputStream of an org.javatuples.Pair whose
classes Pair, Tuple, Object[], Integer, Number, Arrays$ArrayList are the ones
used here; tests/golden/ref_scheduler.ser) and ``ETHModel`` (the ``[D``
descriptor; tests/golden/ref_ethmodel_head.bin).
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC = b"\xac\xed\x00\x05"
TC_NULL, TC_REFERENCE, TC_CLASSDESC, TC_OBJECT, TC_STRING, TC_ARRAY = 0x70, 0x71, 0x72, 0x73, 0x74, 0x75
TC_BLOCKDATA, TC_ENDBLOCKDATA, TC_BLOCKDATALONG, TC_LONGSTRING = 0x77, 0x78, 0x7A, 0x7C
BASE_HANDLE = 0x7E0000
SC_WRITE_METHOD, SC_SERIALIZABLE = 0x01, 0x02

# serialVersionUIDs as they appear in the reference's own serialized files
SUID = {
    "org.javatuples.Pair": 0x21D5DEE583774BBA,          # ref Scheduler
    "org.javatuples.Tuple": 0x4B5F179B83A89E3D,         # ref Scheduler
    "[Ljava.lang.Object;": 0x90CE589F1073296C,          # ref Scheduler
    "java.lang.Integer": 0x12E2A0A4F7818738,            # ref Scheduler
    "java.lang.Number": 0x86AC951D0B94E08B,             # ref Scheduler
    "java.util.Arrays$ArrayList": 0xD9A43CBECD8806D2,   # ref Scheduler
    "[D": 0x3EA68C14AB635A1E,                           # ref ETHModel
}


# ---------------------------------------------------------------------------
# writer: ObjectOutputStream.writeObject(new Pair<>(Integer workers, double[] g))
# ---------------------------------------------------------------------------
class _W:
    def __init__(self):
        self.b = bytearray(MAGIC)
        self.next = BASE_HANDLE

    def handle(self) -> int:
        h = self.next
        self.next += 1
        return h

    def u8(self, v):
        self.b += struct.pack(">B", v)

    def u16(self, v):
        self.b += struct.pack(">H", v)

    def i32(self, v):
        self.b += struct.pack(">i", v)

    def u64(self, v):
        self.b += struct.pack(">Q", v)

    def utf(self, s: str):
        e = s.encode("utf-8")
        self.u16(len(e))
        self.b += e

    def ref(self, h: int):
        self.u8(TC_REFERENCE)
        self.i32(h)


def encode_pair(workers: int, gradients) -> bytes:
    """The bytes ObjectOutputStream writes for new Pair<>(workers, gradients)."""
    g = np.ascontiguousarray(gradients, dtype=np.float64)
    w = _W()
    w.u8(TC_OBJECT)
    # class desc org.javatuples.Pair: fields val0, val1 (Object)
    w.u8(TC_CLASSDESC); w.utf("org.javatuples.Pair"); w.u64(SUID["org.javatuples.Pair"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(2)
    w.u8(ord("L")); w.utf("val0"); w.u8(TC_STRING); w.utf("Ljava/lang/Object;"); h_objsig = w.handle()
    w.u8(ord("L")); w.utf("val1"); w.ref(h_objsig)
    w.u8(TC_ENDBLOCKDATA)
    # superclass org.javatuples.Tuple: fields valueArray (Object[]), valueList (List)
    w.u8(TC_CLASSDESC); w.utf("org.javatuples.Tuple"); w.u64(SUID["org.javatuples.Tuple"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(2)
    w.u8(ord("[")); w.utf("valueArray"); w.u8(TC_STRING); w.utf("[Ljava/lang/Object;"); h_arrsig = w.handle()
    w.u8(ord("L")); w.utf("valueList"); w.u8(TC_STRING); w.utf("Ljava/util/List;"); w.handle()
    w.u8(TC_ENDBLOCKDATA); w.u8(TC_NULL)
    w.handle()                                            # the Pair object
    # Tuple.valueArray = Object[]{workers, gradients}
    w.u8(TC_ARRAY)
    w.u8(TC_CLASSDESC); w.utf("[Ljava.lang.Object;"); w.u64(SUID["[Ljava.lang.Object;"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(0); w.u8(TC_ENDBLOCKDATA); w.u8(TC_NULL)
    h_array = w.handle()
    w.i32(2)
    #   [0] java.lang.Integer(workers) extends java.lang.Number
    w.u8(TC_OBJECT)
    w.u8(TC_CLASSDESC); w.utf("java.lang.Integer"); w.u64(SUID["java.lang.Integer"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(1); w.u8(ord("I")); w.utf("value"); w.u8(TC_ENDBLOCKDATA)
    w.u8(TC_CLASSDESC); w.utf("java.lang.Number"); w.u64(SUID["java.lang.Number"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(0); w.u8(TC_ENDBLOCKDATA); w.u8(TC_NULL)
    h_int = w.handle()
    w.i32(workers)
    #   [1] double[]
    w.u8(TC_ARRAY)
    w.u8(TC_CLASSDESC); w.utf("[D"); w.u64(SUID["[D"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(0); w.u8(TC_ENDBLOCKDATA); w.u8(TC_NULL)
    h_dbl = w.handle()
    w.i32(len(g))
    w.b += g.astype(">f8").tobytes()                     # DataOutput.writeDouble: doubleToLongBits
    # Tuple.valueList = Arrays.asList(valueArray)
    w.u8(TC_OBJECT)
    w.u8(TC_CLASSDESC); w.utf("java.util.Arrays$ArrayList"); w.u64(SUID["java.util.Arrays$ArrayList"]); w.handle()
    w.u8(SC_SERIALIZABLE); w.u16(1); w.u8(ord("[")); w.utf("a"); w.ref(h_arrsig)
    w.u8(TC_ENDBLOCKDATA); w.u8(TC_NULL)
    w.handle()
    w.ref(h_array)
    # Pair.val0, Pair.val1
    w.ref(h_int)
    w.ref(h_dbl)
    return bytes(w.b)


# ---------------------------------------------------------------------------
# reader: the grammar subset (objects, class descs, strings, arrays, refs,
# block data), enough for any stream of serializable non-enum classes
# ---------------------------------------------------------------------------
class JavaFormatError(ValueError):
    pass


_PRIM = {"B": 1, "C": 2, "D": 8, "F": 4, "I": 4, "J": 8, "S": 2, "Z": 1}


class _R:
    def __init__(self, b: bytes):
        self.b = memoryview(b)
        self.i = 0
        self.handles = []

    def take(self, n):
        if n < 0 or self.i + n > len(self.b):
            raise JavaFormatError("truncated stream")
        v = bytes(self.b[self.i:self.i + n])
        self.i += n
        return v

    def u8(self):
        return self.take(1)[0]

    def u16(self):
        return struct.unpack(">H", self.take(2))[0]

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def utf(self):
        return self.take(self.u16()).decode("utf-8", "surrogatepass")

    def assign(self, obj):
        self.handles.append(obj)
        return obj

    def content(self, depth=0):
        if depth > 64:
            raise JavaFormatError("nesting too deep")
        tc = self.u8()
        if tc == TC_NULL:
            return None
        if tc == TC_REFERENCE:
            h = self.i32() - BASE_HANDLE
            if not 0 <= h < len(self.handles):
                raise JavaFormatError("bad handle")
            return self.handles[h]
        if tc == TC_CLASSDESC:
            d = {"kind": "desc", "name": self.utf()}
            d["suid"] = struct.unpack(">Q", self.take(8))[0]
            self.assign(d)
            d["flags"] = self.u8()
            fields = []
            for _ in range(self.u16()):
                t = chr(self.u8())
                name = self.utf()
                if t in "L[":
                    sig = self.content(depth + 1)
                    if not isinstance(sig, str):
                        raise JavaFormatError("field signature is not a string")
                elif t not in _PRIM:
                    raise JavaFormatError(f"bad field type {t!r}")
                fields.append((t, name))
            d["fields"] = fields
            self.annotation(depth)
            d["super"] = self.content(depth + 1)
            if d["super"] is not None and not (isinstance(d["super"], dict) and d["super"].get("kind") == "desc"):
                raise JavaFormatError("superclass is not a class descriptor")
            return d
        if tc in (TC_STRING, TC_LONGSTRING):
            n = self.u16() if tc == TC_STRING else struct.unpack(">Q", self.take(8))[0]
            return self.assign(self.take(n).decode("utf-8", "surrogatepass"))
        if tc == TC_ARRAY:
            desc = self.content(depth + 1)
            if not (isinstance(desc, dict) and desc.get("kind") == "desc" and desc["name"].startswith("[")):
                raise JavaFormatError("array without an array class descriptor")
            a = self.assign({"kind": "array", "desc": desc})
            n = self.i32()
            if n < 0:
                raise JavaFormatError("negative array length")
            et = desc["name"][1]
            if et in _PRIM:
                a["offset"] = self.i
                a["length"] = n
                raw = self.take(n * _PRIM[et])
                if et == "D":
                    a["values"] = np.frombuffer(raw, dtype=">f8").astype(np.float64)
                elif et == "I":
                    a["values"] = np.frombuffer(raw, dtype=">i4").astype(np.int64)
            else:
                a["values"] = [self.content(depth + 1) for _ in range(n)]
            return a
        if tc == TC_OBJECT:
            desc = self.content(depth + 1)
            if not (isinstance(desc, dict) and desc.get("kind") == "desc"):
                raise JavaFormatError("object without a class descriptor")
            o = self.assign({"kind": "object", "class": desc["name"], "fields": {}})
            chain = []
            d = desc
            while d is not None:
                chain.append(d)
                d = d["super"]
            for d in reversed(chain):                   # superclass data first
                if not d["flags"] & SC_SERIALIZABLE or d["flags"] & 0x04:
                    raise JavaFormatError("only Serializable (not Externalizable) classes")
                for t, name in d["fields"]:
                    if t in _PRIM:
                        raw = self.take(_PRIM[t])
                        v = struct.unpack({"B": ">b", "C": ">H", "D": ">d", "F": ">f", "I": ">i", "J": ">q",
                                           "S": ">h", "Z": ">?"}[t], raw)[0]
                    else:
                        v = self.content(depth + 1)
                    o["fields"][(d["name"], name)] = v
                if d["flags"] & SC_WRITE_METHOD:
                    o.setdefault("annotations", {})[d["name"]] = self.annotation(depth)
            return o
        raise JavaFormatError(f"unsupported type code 0x{tc:02x}")

    def annotation(self, depth):
        """Contents up to TC_ENDBLOCKDATA (block data kept as bytes)."""
        items = []
        while True:
            if self.i >= len(self.b):
                raise JavaFormatError("truncated annotation")
            tc = self.b[self.i]
            if tc == TC_ENDBLOCKDATA:
                self.i += 1
                return items
            if tc == TC_BLOCKDATA:
                self.i += 1
                items.append(self.take(self.u8()))
            elif tc == TC_BLOCKDATALONG:
                self.i += 1
                items.append(self.take(self.i32()))
            else:
                items.append(self.content(depth + 1))


def read_object(b: bytes):
    """ObjectInputStream.readObject of the first object of the stream."""
    if bytes(b[:4]) != MAGIC:
        raise JavaFormatError("not an object stream")
    r = _R(b)
    r.i = 4
    return r.content(), r.i


def parse_pair(b: bytes):
    """Download_Partial_Updates (MyIPFSClass.java:326-338): -> (workers,
    gradients, byte offset of the first gradient double)."""
    o, _ = read_object(b)
    if not (isinstance(o, dict) and o.get("class") == "org.javatuples.Pair"):
        raise JavaFormatError("not an org.javatuples.Pair")
    v0 = o["fields"].get(("org.javatuples.Pair", "val0"))
    v1 = o["fields"].get(("org.javatuples.Pair", "val1"))
    if not (isinstance(v0, dict) and v0.get("class") == "java.lang.Integer"):
        raise JavaFormatError("val0 is not an Integer")
    if not (isinstance(v1, dict) and v1.get("kind") == "array" and v1["desc"]["name"] == "[D"):
        raise JavaFormatError("val1 is not a double[]")
    return int(v0["fields"][("java.lang.Integer", "value")]), v1["values"], v1["offset"]
