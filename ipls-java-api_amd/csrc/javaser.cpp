// javaser.cpp -- see javaser.hpp.  The stream grammar is the Java Object
// Serialization Specification's (magic, TC_* tags, class descriptors,
// handles from 0x7e0000); the serialVersionUIDs are the ones in the files the
// reference wrote itself (its Scheduler file: org.javatuples.Pair/Tuple,
// Object[], Integer, Number, Arrays$ArrayList; ETHModel: [D).
#include "javaser.hpp"

#include <cstring>
#include <string>
#include <vector>

namespace ipls {
namespace javaser {
namespace {

constexpr uint8_t TC_NULL = 0x70, TC_REFERENCE = 0x71, TC_CLASSDESC = 0x72, TC_OBJECT = 0x73, TC_STRING = 0x74,
                  TC_ARRAY = 0x75, TC_BLOCKDATA = 0x77, TC_ENDBLOCKDATA = 0x78, TC_BLOCKDATALONG = 0x7A,
                  TC_LONGSTRING = 0x7C;
constexpr uint8_t SC_WRITE_METHOD = 0x01, SC_SERIALIZABLE = 0x02, SC_EXTERNALIZABLE = 0x04;
constexpr int32_t kBaseHandle = 0x7E0000;

constexpr uint64_t kSuidPair = 0x21D5DEE583774BBAull, kSuidTuple = 0x4B5F179B83A89E3Dull,
                   kSuidObjArray = 0x90CE589F1073296Cull, kSuidInteger = 0x12E2A0A4F7818738ull,
                   kSuidNumber = 0x86AC951D0B94E08Bull, kSuidArraysList = 0xD9A43CBECD8806D2ull,
                   kSuidDoubleArray = 0x3EA68C14AB635A1Eull;

// ---- writer ---------------------------------------------------------------
struct Writer {
  uint8_t* p;     // may be null: count only
  int64_t n = 0;
  int32_t next = kBaseHandle;
  void u8(uint8_t v) {
    if (p) p[n] = v;
    ++n;
  }
  void u16(uint16_t v) { u8(uint8_t(v >> 8)), u8(uint8_t(v)); }
  void i32(int32_t v) {
    for (int s = 24; s >= 0; s -= 8) u8(uint8_t(uint32_t(v) >> s));
  }
  void u64(uint64_t v) {
    for (int s = 56; s >= 0; s -= 8) u8(uint8_t(v >> s));
  }
  void utf(const char* s) {   // ASCII class/field names: modified UTF-8 == bytes
    const size_t l = std::strlen(s);
    u16(uint16_t(l));
    for (size_t k = 0; k < l; ++k) u8(uint8_t(s[k]));
  }
  int32_t handle() { return next++; }
  void ref(int32_t h) { u8(TC_REFERENCE), i32(h); }
  // TC_CLASSDESC name suid; the descriptor's handle is assigned here
  int32_t desc(const char* name, uint64_t suid) {
    u8(TC_CLASSDESC), utf(name), u64(suid);
    const int32_t h = handle();
    u8(SC_SERIALIZABLE);
    return h;
  }
};

// Handles the header assigns, in stream order (encode_pair in oracle/javaser.py).
struct PairHandles {
  int32_t obj_sig, arr_sig, array, integer, doubles;
};

PairHandles emit_header(Writer& w, int32_t workers, int32_t n) {
  PairHandles hs{};
  w.u8(0xAC), w.u8(0xED), w.u16(5);   // STREAM_MAGIC, STREAM_VERSION
  w.u8(TC_OBJECT);
  w.desc("org.javatuples.Pair", kSuidPair);
  w.u16(2);
  w.u8('L'), w.utf("val0"), w.u8(TC_STRING), w.utf("Ljava/lang/Object;");
  hs.obj_sig = w.handle();
  w.u8('L'), w.utf("val1"), w.ref(hs.obj_sig);
  w.u8(TC_ENDBLOCKDATA);
  w.desc("org.javatuples.Tuple", kSuidTuple);
  w.u16(2);
  w.u8('['), w.utf("valueArray"), w.u8(TC_STRING), w.utf("[Ljava/lang/Object;");
  hs.arr_sig = w.handle();
  w.u8('L'), w.utf("valueList"), w.u8(TC_STRING), w.utf("Ljava/util/List;");
  w.handle();
  w.u8(TC_ENDBLOCKDATA), w.u8(TC_NULL);
  w.handle();   // the Pair
  // Tuple.valueArray = Object[]{Integer workers, double[] gradients}
  w.u8(TC_ARRAY);
  w.desc("[Ljava.lang.Object;", kSuidObjArray);
  w.u16(0), w.u8(TC_ENDBLOCKDATA), w.u8(TC_NULL);
  hs.array = w.handle();
  w.i32(2);
  w.u8(TC_OBJECT);
  w.desc("java.lang.Integer", kSuidInteger);
  w.u16(1), w.u8('I'), w.utf("value"), w.u8(TC_ENDBLOCKDATA);
  w.desc("java.lang.Number", kSuidNumber);
  w.u16(0), w.u8(TC_ENDBLOCKDATA), w.u8(TC_NULL);
  hs.integer = w.handle();
  w.i32(workers);
  w.u8(TC_ARRAY);
  w.desc("[D", kSuidDoubleArray);
  w.u16(0), w.u8(TC_ENDBLOCKDATA), w.u8(TC_NULL);
  hs.doubles = w.handle();
  w.i32(n);   // then n doubles, DataOutput.writeDouble (big-endian doubleToLongBits)
  return hs;
}

void emit_trailer(Writer& w, const PairHandles& hs) {
  // Tuple.valueList = Arrays.asList(valueArray)
  w.u8(TC_OBJECT);
  w.desc("java.util.Arrays$ArrayList", kSuidArraysList);
  w.u16(1), w.u8('['), w.utf("a"), w.ref(hs.arr_sig);
  w.u8(TC_ENDBLOCKDATA), w.u8(TC_NULL);
  w.handle();
  w.ref(hs.array);
  // Pair.val0, Pair.val1
  w.ref(hs.integer);
  w.ref(hs.doubles);
}

// ---- reader ---------------------------------------------------------------
struct Field {
  char type;
  std::string name;
};

struct Node {
  enum Kind : uint8_t { kDesc, kStr, kObj, kArr } kind;
  std::string name;          // kDesc: class name; kStr: value
  uint8_t flags = 0;         // kDesc
  std::vector<Field> fields; // kDesc
  int super = -1;            // kDesc: superclass handle, -1 = none
  int desc = -1;             // kObj / kArr: class descriptor handle
  struct Val {
    int desc, field;         // which class, which field of it
    int64_t v;               // primitive bits, or a handle (-1 = null) for references
  };
  std::vector<Val> vals;     // kObj
  int64_t len = 0, off = 0;  // kArr of primitives: element count, byte offset of element 0
};

int prim_size(char t) {
  switch (t) {
    case 'B': case 'Z': return 1;
    case 'C': case 'S': return 2;
    case 'I': case 'F': return 4;
    case 'D': case 'J': return 8;
    default: return 0;
  }
}

class Parser {
 public:
  Parser(const uint8_t* b, int64_t n) : b_(b), n_(n) {}
  const char* why = nullptr;
  std::vector<Node> h;

  bool magic() {
    if (n_ < 4 || b_[0] != 0xAC || b_[1] != 0xED || b_[2] != 0x00 || b_[3] != 0x05) return fail("not an object stream");
    i_ = 4;
    return true;
  }
  // -> handle (>= 0), -1 for null, -2 on error
  int content(int depth) {
    if (depth > 64) return fail("nesting too deep"), -2;
    uint8_t tc;
    if (!u8(tc)) return -2;
    switch (tc) {
      case TC_NULL: return -1;
      case TC_REFERENCE: {
        int32_t r;
        if (!i32(r)) return -2;
        const int64_t k = int64_t(r) - kBaseHandle;
        if (k < 0 || k >= (int64_t)h.size()) return fail("bad handle"), -2;
        return int(k);
      }
      case TC_CLASSDESC: return class_desc(depth);
      case TC_STRING:
      case TC_LONGSTRING: {
        int64_t len;
        if (tc == TC_STRING) {
          uint16_t l;
          if (!u16(l)) return -2;
          len = l;
        } else {
          uint64_t l;
          if (!u64(l)) return -2;
          if (l > (uint64_t)n_) return fail("truncated stream"), -2;
          len = int64_t(l);
        }
        if (len > n_ - i_) return fail("truncated stream"), -2;
        Node s{Node::kStr};
        s.name.assign((const char*)b_ + i_, size_t(len));
        i_ += len;
        return assign(std::move(s));
      }
      case TC_ARRAY: return array(depth);
      case TC_OBJECT: return object(depth);
      default: return fail("unsupported type code"), -2;
    }
  }

 private:
  const uint8_t* b_;
  int64_t n_, i_ = 0;

  bool fail(const char* w) {
    if (!why) why = w;
    return false;
  }
  bool need(int64_t k) { return (k >= 0 && k <= n_ - i_) ? true : fail("truncated stream"); }
  bool u8(uint8_t& v) {
    if (!need(1)) return false;
    v = b_[i_++];
    return true;
  }
  bool u16(uint16_t& v) {
    if (!need(2)) return false;
    v = uint16_t(b_[i_] << 8 | b_[i_ + 1]);
    i_ += 2;
    return true;
  }
  bool i32(int32_t& v) {
    if (!need(4)) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; ++k) x = x << 8 | b_[i_ + k];
    i_ += 4;
    v = int32_t(x);
    return true;
  }
  bool u64(uint64_t& v) {
    if (!need(8)) return false;
    v = 0;
    for (int k = 0; k < 8; ++k) v = v << 8 | b_[i_ + k];
    i_ += 8;
    return true;
  }
  bool utf(std::string& s) {
    uint16_t l;
    if (!u16(l) || !need(l)) return false;
    s.assign((const char*)b_ + i_, l);
    i_ += l;
    return true;
  }
  int assign(Node&& x) {
    if (h.size() >= (1u << 22)) return fail("too many objects"), -2;
    h.push_back(std::move(x));
    return int(h.size() - 1);
  }
  bool is_desc(int k) const { return k >= 0 && h[k].kind == Node::kDesc; }

  int class_desc(int depth) {
    Node d{Node::kDesc};
    uint64_t suid;
    if (!utf(d.name) || !u64(suid)) return -2;
    const int me = assign(std::move(d));   // the handle precedes the fields' signature strings
    if (me < 0) return -2;
    uint8_t flags;
    uint16_t nf;
    if (!u8(flags) || !u16(nf)) return -2;
    h[me].flags = flags;
    for (int f = 0; f < nf; ++f) {
      uint8_t t;
      Field fd;
      if (!u8(t) || !utf(fd.name)) return -2;
      fd.type = char(t);
      if (t == 'L' || t == '[') {
        const int sig = content(depth + 1);
        if (sig < 0 || h[sig].kind != Node::kStr) return fail("field signature is not a string"), -2;
      } else if (!prim_size(fd.type)) {
        return fail("bad field type"), -2;
      }
      h[me].fields.push_back(std::move(fd));
    }
    if (!annotation(depth)) return -2;
    const int sup = content(depth + 1);
    if (sup == -2 || (sup >= 0 && !is_desc(sup))) return fail("superclass is not a class descriptor"), -2;
    h[me].super = sup;
    return me;
  }

  bool annotation(int depth) {   // contents up to TC_ENDBLOCKDATA
    for (;;) {
      if (!need(1)) return false;
      const uint8_t tc = b_[i_];
      if (tc == TC_ENDBLOCKDATA) {
        ++i_;
        return true;
      }
      if (tc == TC_BLOCKDATA) {
        ++i_;
        uint8_t l;
        if (!u8(l) || !need(l)) return false;
        i_ += l;
      } else if (tc == TC_BLOCKDATALONG) {
        ++i_;
        int32_t l;
        if (!i32(l) || !need(l)) return false;
        i_ += l;
      } else if (content(depth + 1) == -2) {
        return false;
      }
    }
  }

  int array(int depth) {
    const int d = content(depth + 1);
    if (!is_desc(d) || h[d].name.size() < 2 || h[d].name[0] != '[') return fail("array without an array class"), -2;
    Node a{Node::kArr};
    a.desc = d;
    const int me = assign(std::move(a));
    if (me < 0) return -2;
    int32_t len;
    if (!i32(len)) return -2;
    if (len < 0) return fail("negative array length"), -2;
    const char et = h[d].name[1];
    h[me].len = len;
    if (const int es = prim_size(et)) {
      h[me].off = i_;
      if (!need(int64_t(len) * es)) return -2;
      i_ += int64_t(len) * es;
    } else if (et == 'L' || et == '[') {
      for (int32_t k = 0; k < len; ++k)
        if (content(depth + 1) == -2) return -2;
    } else {
      return fail("bad array class"), -2;
    }
    return me;
  }

  int object(int depth) {
    const int d = content(depth + 1);
    if (!is_desc(d)) return fail("object without a class descriptor"), -2;
    Node o{Node::kObj};
    o.desc = d;
    const int me = assign(std::move(o));
    if (me < 0) return -2;
    std::vector<int> chain;
    for (int c = d; c >= 0; c = h[c].super) {
      if (chain.size() > 64) return fail("class hierarchy too deep"), -2;
      chain.push_back(c);
    }
    for (auto it = chain.rbegin(); it != chain.rend(); ++it) {   // superclass data first
      const int c = *it;
      const uint8_t fl = h[c].flags;
      if (!(fl & SC_SERIALIZABLE) || (fl & SC_EXTERNALIZABLE)) return fail("not a Serializable class"), -2;
      for (size_t f = 0; f < h[c].fields.size(); ++f) {
        const char t = h[c].fields[f].type;
        int64_t v = 0;
        if (const int s = prim_size(t)) {
          if (!need(s)) return -2;
          uint64_t x = 0;
          for (int k = 0; k < s; ++k) x = x << 8 | b_[i_ + k];
          i_ += s;
          v = (s == 4) ? int64_t(int32_t(uint32_t(x))) : int64_t(x);
        } else {
          v = content(depth + 1);
          if (v == -2) return -2;
        }
        h[me].vals.push_back(Node::Val{c, int(f), v});
      }
      if ((fl & SC_WRITE_METHOD) && !annotation(depth)) return -2;
    }
    return me;
  }
};

const Node::Val* field_of(const std::vector<Node>& h, int obj, const char* cls, const char* name) {
  for (const auto& v : h[obj].vals)
    if (h[v.desc].name == cls && h[v.desc].fields[v.field].name == name) return &v;
  return nullptr;
}

}  // namespace

int64_t pair_header_len() {
  Writer w{nullptr};
  emit_header(w, 0, 0);
  return w.n;
}

int64_t pair_trailer_len() {
  Writer w{nullptr};
  const PairHandles hs = emit_header(w, 0, 0);
  Writer t{nullptr};
  t.next = w.next;
  emit_trailer(t, hs);
  return t.n;
}

void write_pair_header(uint8_t* out, int32_t workers, int32_t n) {
  Writer w{out};
  emit_header(w, workers, n);
}

void write_pair_trailer(uint8_t* out) {
  Writer w{nullptr};
  const PairHandles hs = emit_header(w, 0, 0);
  Writer t{out};
  t.next = w.next;
  emit_trailer(t, hs);
}

int64_t parse_pair(const uint8_t* buf, int64_t n, int32_t* workers, int64_t* payload_off, const char** why) {
  Parser ps(buf, n);
  auto bad = [&](const char* w) -> int64_t {
    if (why) *why = ps.why ? ps.why : w;
    return -1;
  };
  if (!buf || !ps.magic()) return bad("not an object stream");
  const int top = ps.content(0);
  if (top < 0) return bad("malformed object stream");
  const auto& h = ps.h;
  if (h[top].kind != Node::kObj || h[h[top].desc].name != "org.javatuples.Pair") return bad("not an org.javatuples.Pair");
  const Node::Val* v0 = field_of(h, top, "org.javatuples.Pair", "val0");
  const Node::Val* v1 = field_of(h, top, "org.javatuples.Pair", "val1");
  if (!v0 || !v1 || v0->v < 0 || v1->v < 0) return bad("Pair without val0/val1");
  const Node& a = h[v0->v];
  const Node& g = h[v1->v];
  if (a.kind != Node::kObj || h[a.desc].name != "java.lang.Integer") return bad("val0 is not an Integer");
  const Node::Val* iv = field_of(h, int(v0->v), "java.lang.Integer", "value");
  if (!iv || h[iv->desc].fields[iv->field].type != 'I') return bad("Integer without an int value");
  if (g.kind != Node::kArr || h[g.desc].name != "[D") return bad("val1 is not a double[]");
  if (workers) *workers = int32_t(iv->v);
  if (payload_off) *payload_off = g.off;
  return g.len;
}

}  // namespace javaser
}  // namespace ipls
