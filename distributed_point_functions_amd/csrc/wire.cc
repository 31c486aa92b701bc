// wire.cc — protobuf wire-format encoding/decoding of the reference's
// messages (dpf/distributed_point_function.proto, pir/
// private_information_retrieval.proto) without a protobuf runtime.  Field
// numbers follow the .proto files; proto3 scalars equal to 0 are omitted,
// oneof members and sub-messages that are set are always written.
#include <string.h>

#include <string>

#include "dpf_amd/protos.h"

namespace distributed_point_functions {
namespace {

// ---------------------------------------------------------------- writer
class Writer {
 public:
  void Varint(uint64_t v) {
    while (v >= 0x80) {
      s_.push_back(static_cast<char>((v & 0x7f) | 0x80));
      v >>= 7;
    }
    s_.push_back(static_cast<char>(v));
  }
  void Tag(int field, int wt) { Varint((static_cast<uint64_t>(field) << 3) | wt); }
  void U64(int field, uint64_t v, bool always = false) {
    if (!v && !always) return;
    Tag(field, 0);
    Varint(v);
  }
  void I32(int field, int32_t v, bool always = false) {
    if (!v && !always) return;
    Tag(field, 0);
    Varint(static_cast<uint64_t>(static_cast<int64_t>(v)));
  }
  void Bool(int field, bool v) {
    if (!v) return;
    Tag(field, 0);
    Varint(1);
  }
  void Double(int field, double v) {
    if (v == 0) return;
    Tag(field, 1);
    char b[8];
    memcpy(b, &v, 8);
    s_.append(b, 8);
  }
  void Bytes(int field, const std::string& v, bool always = false) {
    if (v.empty() && !always) return;
    Tag(field, 2);
    Varint(v.size());
    s_.append(v);
  }
  void Message(int field, const std::string& v) { Bytes(field, v, true); }
  std::string Take() { return std::move(s_); }

 private:
  std::string s_;
};

// ---------------------------------------------------------------- reader
class Reader {
 public:
  Reader(const void* p, size_t n) : p_(static_cast<const uint8_t*>(p)), e_(p_ + n) {}
  bool done() const { return p_ >= e_; }
  bool ok() const { return ok_; }
  bool Next(int* field, int* wt) {
    uint64_t key;
    if (!Varint(&key)) return false;
    *field = static_cast<int>(key >> 3);
    *wt = static_cast<int>(key & 7);
    return *field > 0;
  }
  bool Varint(uint64_t* v) {
    uint64_t r = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p_ >= e_) return Fail();
      uint8_t b = *p_++;
      r |= static_cast<uint64_t>(b & 0x7f) << shift;
      if (!(b & 0x80)) {
        *v = r;
        return true;
      }
    }
    return Fail();
  }
  bool Bytes(const uint8_t** data, size_t* len) {
    uint64_t n;
    if (!Varint(&n) || n > static_cast<uint64_t>(e_ - p_)) return Fail();
    *data = p_;
    *len = static_cast<size_t>(n);
    p_ += n;
    return true;
  }
  bool Fixed64(uint64_t* v) {
    if (e_ - p_ < 8) return Fail();
    memcpy(v, p_, 8);
    p_ += 8;
    return true;
  }
  bool Skip(int wt) {
    uint64_t v;
    const uint8_t* d;
    size_t n;
    switch (wt) {
      case 0:
        return Varint(&v);
      case 1:
        return Fixed64(&v);
      case 2:
        return Bytes(&d, &n);
      case 5:
        if (e_ - p_ < 4) return Fail();
        p_ += 4;
        return true;
      default:
        return Fail();
    }
  }

 private:
  bool Fail() {
    ok_ = false;
    return false;
  }
  const uint8_t* p_;
  const uint8_t* e_;
  bool ok_ = true;
};

#define DPF_FOR_EACH_FIELD(r, f, wt) for (int f, wt; !(r).done() && (r).Next(&f, &wt);)

// --- Block ---
std::string Ser(const Block& b) {
  Writer w;
  w.U64(1, b.high());
  w.U64(2, b.low());
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, Block* b) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    uint64_t v;
    if (f == 1 && wt == 0) {
      if (!r.Varint(&v)) return false;
      b->set_high(v);
    } else if (f == 2 && wt == 0) {
      if (!r.Varint(&v)) return false;
      b->set_low(v);
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

// --- Value ---
std::string Ser(const Value::Integer& i) {
  Writer w;
  if (i.value_case() == Value::Integer::kValueUint64) w.U64(1, i.value_uint64(), true);
  if (i.value_case() == Value::Integer::kValueUint128) w.Message(2, Ser(i.value_uint128()));
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, Value::Integer* i) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    if (f == 1 && wt == 0) {
      uint64_t v;
      if (!r.Varint(&v)) return false;
      i->set_value_uint64(v);
    } else if (f == 2 && wt == 2) {
      const uint8_t* d;
      size_t l;
      if (!r.Bytes(&d, &l) || !Par(d, l, i->mutable_value_uint128())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string Ser(const Value& v) {
  Writer w;
  switch (v.value_case()) {
    case Value::kInteger:
      w.Message(1, Ser(v.integer()));
      break;
    case Value::kTuple: {
      Writer t;
      for (const Value& e : v.tuple().elements()) t.Message(1, Ser(e));
      w.Message(2, t.Take());
      break;
    }
    case Value::kIntModN:
      w.Message(3, Ser(v.int_mod_n()));
      break;
    case Value::kXorWrapper:
      w.Message(4, Ser(v.xor_wrapper()));
      break;
    default:
      break;
  }
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, Value* v, int depth = 0) {
  if (depth > 32) return false;
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (wt != 2) {
      if (!r.Skip(wt)) return false;
      continue;
    }
    if (!r.Bytes(&d, &l)) return false;
    bool ok = true;
    if (f == 1) {
      ok = Par(d, l, v->mutable_integer());
    } else if (f == 2) {
      Value::Tuple* t = v->mutable_tuple();
      Reader tr(d, l);
      DPF_FOR_EACH_FIELD(tr, tf, twt) {
        if (tf == 1 && twt == 2) {
          const uint8_t* ed;
          size_t el;
          if (!tr.Bytes(&ed, &el) || !Par(ed, el, t->add_elements(), depth + 1)) return false;
        } else if (!tr.Skip(twt)) {
          return false;
        }
      }
      ok = tr.ok();
    } else if (f == 3) {
      ok = Par(d, l, v->mutable_int_mod_n());
    } else if (f == 4) {
      ok = Par(d, l, v->mutable_xor_wrapper());
    }
    if (!ok) return false;
  }
  return r.ok();
}

// --- ValueType ---
std::string Ser(const ValueType::Integer& i) {
  Writer w;
  w.I32(1, i.bitsize());
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, ValueType::Integer* i) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    if (f == 1 && wt == 0) {
      uint64_t v;
      if (!r.Varint(&v)) return false;
      i->set_bitsize(static_cast<int32_t>(v));
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string Ser(const ValueType& vt) {
  Writer w;
  switch (vt.type_case()) {
    case ValueType::kInteger:
      w.Message(1, Ser(vt.integer()));
      break;
    case ValueType::kTuple: {
      Writer t;
      for (const ValueType& e : vt.tuple().elements()) t.Message(1, Ser(e));
      w.Message(2, t.Take());
      break;
    }
    case ValueType::kIntModN: {
      Writer m;
      if (vt.int_mod_n().has_base_integer())
        m.Message(1, Ser(vt.int_mod_n().base_integer()));
      if (vt.int_mod_n().has_modulus()) m.Message(2, Ser(vt.int_mod_n().modulus()));
      w.Message(3, m.Take());
      break;
    }
    case ValueType::kXorWrapper:
      w.Message(4, Ser(vt.xor_wrapper()));
      break;
    default:
      break;
  }
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, ValueType* vt, int depth = 0) {
  if (depth > 32) return false;
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (wt != 2) {
      if (!r.Skip(wt)) return false;
      continue;
    }
    if (!r.Bytes(&d, &l)) return false;
    bool ok = true;
    if (f == 1) {
      ok = Par(d, l, vt->mutable_integer());
    } else if (f == 2) {
      ValueType::Tuple* t = vt->mutable_tuple();
      Reader tr(d, l);
      DPF_FOR_EACH_FIELD(tr, tf, twt) {
        if (tf == 1 && twt == 2) {
          const uint8_t* ed;
          size_t el;
          if (!tr.Bytes(&ed, &el) || !Par(ed, el, t->add_elements(), depth + 1)) return false;
        } else if (!tr.Skip(twt)) {
          return false;
        }
      }
      ok = tr.ok();
    } else if (f == 3) {
      ValueType::IntModN* m = vt->mutable_int_mod_n();
      Reader mr(d, l);
      DPF_FOR_EACH_FIELD(mr, mf, mwt) {
        const uint8_t* md;
        size_t ml;
        if (mwt == 2 && (mf == 1 || mf == 2)) {
          if (!mr.Bytes(&md, &ml)) return false;
          if (mf == 1 && !Par(md, ml, m->mutable_base_integer())) return false;
          if (mf == 2 && !Par(md, ml, m->mutable_modulus())) return false;
        } else if (!mr.Skip(mwt)) {
          return false;
        }
      }
      ok = mr.ok();
    } else if (f == 4) {
      ok = Par(d, l, vt->mutable_xor_wrapper());
    }
    if (!ok) return false;
  }
  return r.ok();
}

// --- DpfParameters ---
std::string Ser(const DpfParameters& p) {
  Writer w;
  w.I32(1, p.log_domain_size());
  if (p.has_value_type()) w.Message(3, Ser(p.value_type()));
  w.Double(4, p.security_parameter());
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, DpfParameters* out) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    if (f == 1 && wt == 0) {
      uint64_t v;
      if (!r.Varint(&v)) return false;
      out->set_log_domain_size(static_cast<int32_t>(v));
    } else if (f == 3 && wt == 2) {
      const uint8_t* d;
      size_t l;
      if (!r.Bytes(&d, &l) || !Par(d, l, out->mutable_value_type())) return false;
    } else if (f == 4 && wt == 1) {
      uint64_t v;
      if (!r.Fixed64(&v)) return false;
      double x;
      memcpy(&x, &v, 8);
      out->set_security_parameter(x);
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

// --- CorrectionWord / DpfKey ---
std::string Ser(const CorrectionWord& c) {
  Writer w;
  if (c.has_seed()) w.Message(1, Ser(c.seed()));
  w.Bool(2, c.control_left());
  w.Bool(3, c.control_right());
  for (const Value& v : c.value_correction()) w.Message(5, Ser(v));
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, CorrectionWord* c) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    uint64_t v;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, c->mutable_seed())) return false;
    } else if ((f == 2 || f == 3) && wt == 0) {
      if (!r.Varint(&v)) return false;
      if (f == 2)
        c->set_control_left(v != 0);
      else
        c->set_control_right(v != 0);
    } else if (f == 5 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, c->add_value_correction())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string Ser(const DpfKey& k) {
  Writer w;
  if (k.has_seed()) w.Message(1, Ser(k.seed()));
  for (const CorrectionWord& c : k.correction_words()) w.Message(2, Ser(c));
  w.I32(3, k.party());
  for (const Value& v : k.last_level_value_correction()) w.Message(5, Ser(v));
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, DpfKey* k) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    uint64_t v;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, k->mutable_seed())) return false;
    } else if (f == 2 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, k->add_correction_words())) return false;
    } else if (f == 3 && wt == 0) {
      if (!r.Varint(&v)) return false;
      k->set_party(static_cast<int32_t>(v));
    } else if (f == 5 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, k->add_last_level_value_correction())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

// --- PartialEvaluation / EvaluationContext ---
std::string Ser(const PartialEvaluation& e) {
  Writer w;
  if (e.has_prefix()) w.Message(1, Ser(e.prefix()));
  if (e.has_seed()) w.Message(2, Ser(e.seed()));
  w.Bool(3, e.control_bit());
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, PartialEvaluation* e) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    uint64_t v;
    if ((f == 1 || f == 2) && wt == 2) {
      if (!r.Bytes(&d, &l)) return false;
      if (!Par(d, l, f == 1 ? e->mutable_prefix() : e->mutable_seed())) return false;
    } else if (f == 3 && wt == 0) {
      if (!r.Varint(&v)) return false;
      e->set_control_bit(v != 0);
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string Ser(const EvaluationContext& c) {
  Writer w;
  for (const DpfParameters& p : c.parameters()) w.Message(1, Ser(p));
  if (c.has_key()) w.Message(2, Ser(c.key()));
  w.I32(3, c.previous_hierarchy_level());
  for (const PartialEvaluation& e : c.partial_evaluations()) w.Message(4, Ser(e));
  w.I32(5, c.partial_evaluations_level());
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, EvaluationContext* c) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    uint64_t v;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, c->add_parameters())) return false;
    } else if (f == 2 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, c->mutable_key())) return false;
    } else if (f == 3 && wt == 0) {
      if (!r.Varint(&v)) return false;
      c->set_previous_hierarchy_level(static_cast<int32_t>(v));
    } else if (f == 4 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, c->add_partial_evaluations())) return false;
    } else if (f == 5 && wt == 0) {
      if (!r.Varint(&v)) return false;
      c->set_partial_evaluations_level(static_cast<int32_t>(v));
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

// --- PIR ---
std::string Ser(const DpfPirRequest::PlainRequest& pr) {
  Writer w;
  for (const DpfKey& k : pr.dpf_key()) w.Message(1, Ser(k));
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, DpfPirRequest::PlainRequest* pr) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, pr->add_dpf_key())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string Ser(const DpfPirRequest::EncryptedHelperRequest& e) {
  Writer w;
  w.Bytes(1, e.encrypted_request());
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, DpfPirRequest::EncryptedHelperRequest* e) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l)) return false;
      e->set_encrypted_request(std::string(reinterpret_cast<const char*>(d), l));
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string Ser(const DpfPirRequest& q) {
  Writer w;
  switch (q.wrapped_request_case()) {
    case DpfPirRequest::kPlainRequest:
      w.Message(1, Ser(q.plain_request()));
      break;
    case DpfPirRequest::kLeaderRequest: {
      Writer l;
      if (q.leader_request().has_plain_request())
        l.Message(1, Ser(q.leader_request().plain_request()));
      if (q.leader_request().has_encrypted_helper_request())
        l.Message(2, Ser(q.leader_request().encrypted_helper_request()));
      w.Message(2, l.Take());
      break;
    }
    case DpfPirRequest::kEncryptedHelperRequest:
      w.Message(3, Ser(q.encrypted_helper_request()));
      break;
    default:
      break;
  }
  return w.Take();
}
bool Par(const uint8_t* p, size_t n, DpfPirRequest* q) {
  Reader r(p, n);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (wt != 2) {
      if (!r.Skip(wt)) return false;
      continue;
    }
    if (!r.Bytes(&d, &l)) return false;
    bool ok = true;
    if (f == 1) {
      ok = Par(d, l, q->mutable_plain_request());
    } else if (f == 2) {
      DpfPirRequest::LeaderRequest* lr = q->mutable_leader_request();
      Reader lrr(d, l);
      DPF_FOR_EACH_FIELD(lrr, lf, lwt) {
        const uint8_t* ld;
        size_t ll;
        if (lwt == 2 && (lf == 1 || lf == 2)) {
          if (!lrr.Bytes(&ld, &ll)) return false;
          if (lf == 1 && !Par(ld, ll, lr->mutable_plain_request())) return false;
          if (lf == 2 && !Par(ld, ll, lr->mutable_encrypted_helper_request())) return false;
        } else if (!lrr.Skip(lwt)) {
          return false;
        }
      }
      ok = lrr.ok();
    } else if (f == 3) {
      ok = Par(d, l, q->mutable_encrypted_helper_request());
    }
    if (!ok) return false;
  }
  return r.ok();
}

}  // namespace

std::string DpfKey::SerializeAsString() const { return Ser(*this); }
bool DpfKey::ParseFromString(const std::string& s) { return ParseFromArray(s.data(), s.size()); }
bool DpfKey::ParseFromArray(const void* data, size_t size) {
  *this = DpfKey();
  return Par(static_cast<const uint8_t*>(data), size, this);
}

std::string EvaluationContext::SerializeAsString() const { return Ser(*this); }
bool EvaluationContext::ParseFromString(const std::string& s) {
  return ParseFromArray(s.data(), s.size());
}
bool EvaluationContext::ParseFromArray(const void* data, size_t size) {
  *this = EvaluationContext();
  return Par(static_cast<const uint8_t*>(data), size, this);
}

// --- DcfParameters / DcfKey (dcf/distributed_comparison_function.proto) ---
std::string DcfParameters::SerializeAsString() const {
  Writer w;
  if (has_parameters()) w.Message(1, Ser(parameters()));
  return w.Take();
}
bool DcfParameters::ParseFromArray(const void* data, size_t size) {
  *this = DcfParameters();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, mutable_parameters())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}
std::string DcfKey::SerializeAsString() const {
  Writer w;
  if (has_key()) w.Message(1, Ser(key()));
  return w.Take();
}
bool DcfKey::ParseFromArray(const void* data, size_t size) {
  *this = DcfKey();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, mutable_key())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

// --- pir/hashing/hash_family_config.proto, CuckooHashingParams ---
std::string HashFamilyConfig::SerializeAsString() const {
  Writer w;
  w.U64(1, static_cast<uint64_t>(static_cast<int64_t>(hash_family_)));
  w.Bytes(2, seed_);
  return w.Take();
}
bool HashFamilyConfig::ParseFromArray(const void* data, size_t size) {
  *this = HashFamilyConfig();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    uint64_t v;
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 0) {
      if (!r.Varint(&v)) return false;
      hash_family_ = static_cast<int>(v);
    } else if (f == 2 && wt == 2) {
      if (!r.Bytes(&d, &l)) return false;
      seed_.assign(reinterpret_cast<const char*>(d), l);
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string CuckooHashingParams::SerializeAsString() const {
  Writer w;
  if (has_hash_family_config_) w.Message(1, hash_family_config_.SerializeAsString());
  w.U64(2, static_cast<uint64_t>(static_cast<int64_t>(num_hash_functions_)));
  w.U64(3, static_cast<uint64_t>(num_buckets_));
  return w.Take();
}
bool CuckooHashingParams::ParseFromArray(const void* data, size_t size) {
  *this = CuckooHashingParams();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    uint64_t v;
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !mutable_hash_family_config()->ParseFromArray(d, l)) return false;
    } else if (f == 2 && wt == 0) {
      if (!r.Varint(&v)) return false;
      num_hash_functions_ = static_cast<int32_t>(v);
    } else if (f == 3 && wt == 0) {
      if (!r.Varint(&v)) return false;
      num_buckets_ = static_cast<int64_t>(v);
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string PirServerPublicParams::SerializeAsString() const {
  Writer w;
  if (case_ == kCuckooHashingSparseDpfPirServerParams) w.Message(1, cuckoo_.SerializeAsString());
  return w.Take();
}
bool PirServerPublicParams::ParseFromArray(const void* data, size_t size) {
  *this = PirServerPublicParams();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) ||
          !mutable_cuckoo_hashing_sparse_dpf_pir_server_params()->ParseFromArray(d, l))
        return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string PirConfig::SerializeAsString() const {
  Writer w;
  if (case_ == kDenseDpfPirConfig) {
    Writer d;
    d.U64(1, static_cast<uint64_t>(dense_.num_elements()));
    w.Message(1, d.Take());
  } else if (case_ == kCuckooHashingSparseDpfPirConfig) {
    Writer d;
    d.U64(1, static_cast<uint64_t>(static_cast<int64_t>(cuckoo_.hash_family())));
    d.U64(2, static_cast<uint64_t>(cuckoo_.num_elements()));
    w.Message(2, d.Take());
  }
  return w.Take();
}
bool PirConfig::ParseFromArray(const void* data, size_t size) {
  *this = PirConfig();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if ((f == 1 || f == 2) && wt == 2) {
      if (!r.Bytes(&d, &l)) return false;
      Reader cr(d, l);
      if (f == 1) mutable_dense_dpf_pir_config();
      else mutable_cuckoo_hashing_sparse_dpf_pir_config();
      DPF_FOR_EACH_FIELD(cr, cf, cwt) {
        uint64_t v;
        if (cwt == 0 && (cf == 1 || (f == 2 && cf == 2))) {
          if (!cr.Varint(&v)) return false;
          if (f == 1) dense_.set_num_elements(static_cast<int64_t>(v));
          else if (cf == 1) cuckoo_.set_hash_family(static_cast<int>(v));
          else cuckoo_.set_num_elements(static_cast<int64_t>(v));
        } else if (!cr.Skip(cwt)) {
          return false;
        }
      }
      if (!cr.ok()) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string PirRequest::SerializeAsString() const {
  Writer w;
  if (case_ == kDpfPirRequest) w.Message(1, Ser(req_));
  return w.Take();
}
bool PirRequest::ParseFromArray(const void* data, size_t size) {
  *this = PirRequest();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, mutable_dpf_pir_request())) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string DpfPirRequest::HelperRequest::SerializeAsString() const {
  Writer w;
  if (has_plain_request_) w.Message(1, Ser(plain_request_));
  w.Bytes(2, one_time_pad_seed_);
  return w.Take();
}
bool DpfPirRequest::HelperRequest::ParseFromString(const std::string& s) {
  *this = HelperRequest();
  Reader r(s.data(), s.size());
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l) || !Par(d, l, mutable_plain_request())) return false;
    } else if (f == 2 && wt == 2) {
      if (!r.Bytes(&d, &l)) return false;
      one_time_pad_seed_.assign(reinterpret_cast<const char*>(d), l);
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

std::string PirResponse::SerializeAsString() const {
  Writer w;
  if (case_ == kDpfPirResponse) {
    Writer d;
    for (const std::string& s : resp_.masked_response()) d.Bytes(1, s, true);
    w.Message(1, d.Take());
  }
  return w.Take();
}
bool PirResponse::ParseFromArray(const void* data, size_t size) {
  *this = PirResponse();
  Reader r(data, size);
  DPF_FOR_EACH_FIELD(r, f, wt) {
    const uint8_t* d;
    size_t l;
    if (f == 1 && wt == 2) {
      if (!r.Bytes(&d, &l)) return false;
      DpfPirResponse* resp = mutable_dpf_pir_response();
      Reader rr(d, l);
      DPF_FOR_EACH_FIELD(rr, rf, rwt) {
        const uint8_t* md;
        size_t ml;
        if (rf == 1 && rwt == 2) {
          if (!rr.Bytes(&md, &ml)) return false;
          resp->add_masked_response()->assign(reinterpret_cast<const char*>(md), ml);
        } else if (!rr.Skip(rwt)) {
          return false;
        }
      }
      if (!rr.ok()) return false;
    } else if (!r.Skip(wt)) {
      return false;
    }
  }
  return r.ok();
}

const PirServerPublicParams& PirServerPublicParams::default_instance() {
  static const PirServerPublicParams k;
  return k;
}

std::string SerializeValueType(const ValueType& vt) { return Ser(vt); }
bool ParseValueType(const void* data, size_t size, ValueType* out) {
  *out = ValueType();
  return Par(static_cast<const uint8_t*>(data), size, out);
}
std::string SerializeValue(const Value& v) { return Ser(v); }
bool ParseValue(const void* data, size_t size, Value* out) {
  *out = Value();
  return Par(static_cast<const uint8_t*>(data), size, out);
}
std::string SerializeDpfParameters(const DpfParameters& p) { return Ser(p); }
bool ParseDpfParameters(const void* data, size_t size, DpfParameters* out) {
  *out = DpfParameters();
  return Par(static_cast<const uint8_t*>(data), size, out);
}

std::string Status::ToString() const {
  static const char* names[] = {"OK", "", "", "INVALID_ARGUMENT", "", "", "", "",
                                "RESOURCE_EXHAUSTED", "FAILED_PRECONDITION", "", "",
                                "UNIMPLEMENTED", "INTERNAL"};
  int c = raw_code();
  std::string n = (c >= 0 && c <= 13 && names[c][0]) ? names[c] : std::to_string(c);
  return ok() ? "OK" : n + ": " + message_;
}

}  // namespace distributed_point_functions
