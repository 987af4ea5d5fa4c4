// codecs.cpp -- reference codecs (codecs.go:15-93) with Go encoding/json and
// regexp behaviour:
//   * JSON in: json.Decoder.Decode into PartitionList (case-insensitive field
//     match, unknown fields ignored, ints must be integer literals, first type
//     error wins, syntax errors first), then the version==1 check (codecs.go:24-26)
//   * text in: `kafka-topics.sh --describe` lines matched by
//     ^\tTopic: ([^\t]*)\tPartition: ([0-9]*)\tLeader: ([0-9]*)\tReplicas: ([0-9,]*)\tIsr: ([0-9,]*)
//     with Atoi errors ignored (codecs.go:28-56), bufio.Scanner 64 KiB lines
//   * JSON out: Go encoding/json bytes (HTML-escaped strings, omitempty,
//     shortest float formatting), trailing newline (json.Encoder)
#include "codecs.hpp"

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <set>
#include <thread>
#include <utility>

namespace kbh {

std::string Partition::str() const {
    std::string s = "Partition(" + topic + "," + std::to_string((long long)partition) + ",[";
    for (size_t i = 0; i < replicas.len; i++) {
        if (i) s += " ";
        s += std::to_string((long long)replicas.at(i));
    }
    return s + "])";
}

// ------------------------------------------------------------ floats

static void shortest(double x, std::string& digits, int& e10) {
    // shortest round-trip digits d1.d2d3... x 10^e10
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, std::fabs(x), std::chars_format::scientific);
    std::string t(buf, r.ptr);
    size_t epos = t.find('e');
    std::string m = t.substr(0, epos);
    e10 = std::atoi(t.c_str() + epos + 1);
    digits.clear();
    for (char c : m) if (c != '.') digits += c;
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
}

// Go encoding/json float64 text appended to o (strconv 'f' / -1, 'e' outside
// [1e-6, 1e21) with a negative exponent's leading zero removed)
void GoFloatAppend(std::string& o, double x) {
    if (x == 0) { o += std::signbit(x) ? "-0" : "0"; return; }
    char buf[40];
    auto r = std::to_chars(buf, buf + sizeof buf, std::fabs(x), std::chars_format::scientific);
    // shortest round-trip digits d[0..nd) and decimal exponent e10 of d[0]
    char d[24];
    int nd = 0;
    const char* q = buf;
    for (; q < r.ptr && *q != 'e'; q++) if (*q != '.') d[nd++] = *q;
    while (nd > 1 && d[nd - 1] == '0') nd--;
    int e10 = 0;
    std::from_chars(q + 1 + (q[1] == '+' ? 1 : 0), r.ptr, e10);
    if (x < 0) o += '-';
    const double a = std::fabs(x);
    if (a < 1e-6 || a >= 1e21) {
        o += d[0];
        if (nd > 1) { o += '.'; o.append(d + 1, (size_t)(nd - 1)); }
        o += 'e';
        if (e10 < 0) { o += '-'; e10 = -e10; }              // e-07 -> e-7 (Go's cleanup)
        else { o += '+'; if (e10 < 10) o += '0'; }
        char eb[8];
        auto er = std::to_chars(eb, eb + sizeof eb, e10);
        o.append(eb, er.ptr);
        return;
    }
    const int point = e10 + 1;
    if (point <= 0) { o += "0."; o.append((size_t)-point, '0'); o.append(d, (size_t)nd); }
    else if (point >= nd) { o.append(d, (size_t)nd); o.append((size_t)(point - nd), '0'); }
    else { o.append(d, (size_t)point); o += '.'; o.append(d + point, (size_t)(nd - point)); }
}

std::string GoFloat(double x) {
    std::string o;
    GoFloatAppend(o, x);
    return o;
}

std::string GoFloatG(double x) {
    if (x == 0) return std::signbit(x) ? "-0" : "0";
    if (std::isinf(x)) return x > 0 ? "+Inf" : "-Inf";
    if (std::isnan(x)) return "NaN";
    std::string d;
    int e10;
    shortest(x, d, e10);
    std::string o = x < 0 ? "-" : "";
    int exp = e10;
    if (exp < -4 || exp >= 21) {
        o += d[0];
        if (d.size() > 1) o += "." + d.substr(1);
        char eb[16];
        snprintf(eb, sizeof eb, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
        return o + eb;
    }
    int point = e10 + 1;
    if (point <= 0) o += "0." + std::string((size_t)-point, '0') + d;
    else if (point >= (int)d.size()) o += d + std::string((size_t)(point - (int)d.size()), '0');
    else o += d.substr(0, (size_t)point) + "." + d.substr((size_t)point);
    return o;
}

// ------------------------------------------------------- JSON parsing

namespace {

struct JVal {
    enum Kind { OBJ, ARR, STR, NUM, BOOL, NUL } k = NUL;
    std::string s;                                   // string value / number literal
    bool b = false;
    std::vector<std::pair<std::string, JVal>> obj;
    std::vector<JVal> arr;
};

std::string quote_char(unsigned char c) {
    if (c == '\'') return "'\\''";
    if (c == '"') return "'\"'";
    if (c >= 0x20 && c < 0x7f) return std::string("'") + (char)c + "'";
    char b[16];
    switch (c) {
        case '\n': return "'\\n'";
        case '\r': return "'\\r'";
        case '\t': return "'\\t'";
        default: snprintf(b, sizeof b, "'\\x%02x'", c); return b;
    }
}

struct Parser {
    const std::string& in;
    size_t i = 0;
    std::string err;
    explicit Parser(const std::string& s) : in(s) {}

    void ws() { while (i < in.size() && (in[i] == ' ' || in[i] == '\t' || in[i] == '\n' || in[i] == '\r')) i++; }
    bool fail(const std::string& m) { if (err.empty()) err = m; return false; }
    bool eof_mid() { return fail("unexpected EOF"); }

    bool value(JVal& v, const char* ctx) {
        ws();
        if (i >= in.size()) return eof_mid();
        char c = in[i];
        if (c == '{') return object(v);
        if (c == '[') return array(v);
        if (c == '"') { v.k = JVal::STR; return str(v.s); }
        if (c == '-' || (c >= '0' && c <= '9')) return number(v);
        if (c == 't') return literal(v, "true", JVal::BOOL, true);
        if (c == 'f') return literal(v, "false", JVal::BOOL, false);
        if (c == 'n') return literal(v, "null", JVal::NUL, false);
        return fail("invalid character " + quote_char((unsigned char)c) + " " + ctx);
    }
    bool literal(JVal& v, const char* lit, JVal::Kind k, bool b) {
        size_t n = strlen(lit);
        for (size_t j = 0; j < n; j++) {
            if (i + j >= in.size()) return eof_mid();
            if (in[i + j] != lit[j])
                return fail("invalid character " + quote_char((unsigned char)in[i + j]) + " in literal " +
                            lit + " (expecting " + quote_char((unsigned char)lit[j]) + ")");
        }
        i += n;
        v.k = k;
        v.b = b;
        return true;
    }
    bool number(JVal& v) {
        size_t st = i;
        if (in[i] == '-') i++;
        if (i >= in.size()) return eof_mid();
        if (in[i] == '0') i++;
        else if (in[i] >= '1' && in[i] <= '9') { while (i < in.size() && isdigit((unsigned char)in[i])) i++; }
        else return fail("invalid character " + quote_char((unsigned char)in[i]) + " in numeric literal");
        if (i < in.size() && in[i] == '.') {
            i++;
            if (i >= in.size()) return eof_mid();
            if (!isdigit((unsigned char)in[i])) return fail("invalid character " + quote_char((unsigned char)in[i]) + " after decimal point in numeric literal");
            while (i < in.size() && isdigit((unsigned char)in[i])) i++;
        }
        if (i < in.size() && (in[i] == 'e' || in[i] == 'E')) {
            i++;
            if (i < in.size() && (in[i] == '+' || in[i] == '-')) i++;
            if (i >= in.size()) return eof_mid();
            if (!isdigit((unsigned char)in[i])) return fail("invalid character " + quote_char((unsigned char)in[i]) + " in exponent of numeric literal");
            while (i < in.size() && isdigit((unsigned char)in[i])) i++;
        }
        v.k = JVal::NUM;
        v.s = in.substr(st, i - st);
        return true;
    }
    static void put_utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
        else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
        else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
    }
    bool hex4(uint32_t& v) {
        v = 0;
        for (int j = 0; j < 4; j++) {
            if (i >= in.size()) return eof_mid();
            char c = in[i++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else return fail("invalid character " + quote_char((unsigned char)c) + " in \\u hexadecimal character escape");
        }
        return true;
    }
    bool str(std::string& o) {
        i++;  // opening quote
        o.clear();
        for (;;) {
            if (i >= in.size()) return eof_mid();
            unsigned char c = (unsigned char)in[i];
            if (c == '"') { i++; return true; }
            if (c < 0x20) return fail("invalid character " + quote_char(c) + " in string literal");
            if (c == '\\') {
                i++;
                if (i >= in.size()) return eof_mid();
                char e = in[i++];
                switch (e) {
                    case '"': o += '"'; break;
                    case '\\': o += '\\'; break;
                    case '/': o += '/'; break;
                    case 'b': o += '\b'; break;
                    case 'f': o += '\f'; break;
                    case 'n': o += '\n'; break;
                    case 'r': o += '\r'; break;
                    case 't': o += '\t'; break;
                    case 'u': {
                        uint32_t cp;
                        if (!hex4(cp)) return false;
                        if (cp >= 0xD800 && cp < 0xDC00 && i + 1 < in.size() && in[i] == '\\' && in[i + 1] == 'u') {
                            size_t save = i;
                            i += 2;
                            uint32_t lo;
                            if (!hex4(lo)) return false;
                            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                            else { i = save; cp = 0xFFFD; }
                        } else if (cp >= 0xD800 && cp < 0xE000) {
                            cp = 0xFFFD;
                        }
                        put_utf8(o, cp);
                        break;
                    }
                    default:
                        return fail("invalid character " + quote_char((unsigned char)e) + " in string escape code");
                }
                continue;
            }
            o += (char)c;
            i++;
        }
    }
    bool object(JVal& v) {
        v.k = JVal::OBJ;
        i++;
        ws();
        if (i >= in.size()) return eof_mid();
        if (in[i] == '}') { i++; return true; }
        for (;;) {
            ws();
            if (i >= in.size()) return eof_mid();
            if (in[i] != '"') return fail("invalid character " + quote_char((unsigned char)in[i]) + " looking for beginning of object key string");
            std::string key;
            if (!str(key)) return false;
            ws();
            if (i >= in.size()) return eof_mid();
            if (in[i] != ':') return fail("invalid character " + quote_char((unsigned char)in[i]) + " after object key");
            i++;
            JVal val;
            if (!value(val, "looking for beginning of value")) return false;
            v.obj.emplace_back(std::move(key), std::move(val));
            ws();
            if (i >= in.size()) return eof_mid();
            if (in[i] == ',') { i++; continue; }
            if (in[i] == '}') { i++; return true; }
            return fail("invalid character " + quote_char((unsigned char)in[i]) + " after object key:value pair");
        }
    }
    bool array(JVal& v) {
        v.k = JVal::ARR;
        i++;
        ws();
        if (i >= in.size()) return eof_mid();
        if (in[i] == ']') { i++; return true; }
        for (;;) {
            JVal el;
            if (!value(el, "looking for beginning of value")) return false;
            v.arr.push_back(std::move(el));
            ws();
            if (i >= in.size()) return eof_mid();
            if (in[i] == ',') { i++; continue; }
            if (in[i] == ']') { i++; return true; }
            return fail("invalid character " + quote_char((unsigned char)in[i]) + " after array element");
        }
    }
};

const char* kind_name(const JVal& v) {
    switch (v.k) {
        case JVal::OBJ: return "object";
        case JVal::ARR: return "array";
        case JVal::STR: return "string";
        case JVal::NUM: return "number";
        case JVal::BOOL: return "bool";
        default: return "null";
    }
}

bool fold_eq(const std::string& a, const char* b) {
    size_t n = strlen(b);
    if (a.size() != n) return false;
    for (size_t i = 0; i < n; i++) if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
    return true;
}

struct Decoder {
    std::string err;   // first UnmarshalTypeError
    void type_err(const JVal& v, const std::string& field, const std::string& type) {
        if (!err.empty()) return;
        std::string what = kind_name(v);
        if (v.k == JVal::NUM) what += " " + v.s;
        err = "json: cannot unmarshal " + what + " into Go struct field " + field + " of type " + type;
    }
    void to_int(const JVal& v, int64_t& out, const std::string& field, const std::string& type) {
        if (v.k == JVal::NUL) return;
        if (v.k != JVal::NUM) return type_err(v, field, type);
        const char* s = v.s.c_str();
        errno = 0;
        char* end = nullptr;
        long long x = strtoll(s, &end, 10);
        if (errno || *end) return type_err(v, field, type);
        out = x;
    }
    void to_float(const JVal& v, double& out, const std::string& field) {
        if (v.k == JVal::NUL) return;
        if (v.k != JVal::NUM) return type_err(v, field, "float64");
        errno = 0;
        double x = strtod(v.s.c_str(), nullptr);
        if (errno == ERANGE && std::isinf(x)) return type_err(v, field, "float64");
        out = x;
    }
    void to_ints(const JVal& v, Slice& out, const std::string& field, const std::string& elem) {
        if (v.k == JVal::NUL) { out = Slice(); return; }
        if (v.k != JVal::ARR) return type_err(v, field, "[]" + elem);
        std::vector<int64_t> xs;
        for (const JVal& e : v.arr) {
            int64_t x = 0;
            to_int(e, x, field, elem);
            xs.push_back(x);
        }
        out = Slice::of(xs);
    }
    void partition(const JVal& v, Partition& p) {
        if (v.k == JVal::NUL) return;
        if (v.k != JVal::OBJ) return type_err(v, "PartitionList.partitions", "main.Partition");
        for (const auto& kv : v.obj) {
            const std::string& k = kv.first;
            const JVal& x = kv.second;
            if (fold_eq(k, "topic")) {
                if (x.k == JVal::NUL) continue;
                if (x.k != JVal::STR) type_err(x, "Partition.partitions.topic", "main.TopicName");
                else p.topic = x.s;
            } else if (fold_eq(k, "partition")) {
                to_int(x, p.partition, "Partition.partitions.partition", "main.PartitionID");
            } else if (fold_eq(k, "replicas")) {
                to_ints(x, p.replicas, "Partition.partitions.replicas", "main.BrokerID");
            } else if (fold_eq(k, "weight")) {
                to_float(x, p.weight, "Partition.partitions.weight");
            } else if (fold_eq(k, "num_replicas")) {
                to_int(x, p.num_replicas, "Partition.partitions.num_replicas", "int");
            } else if (fold_eq(k, "brokers")) {
                to_ints(x, p.brokers, "Partition.partitions.brokers", "main.BrokerID");
            } else if (fold_eq(k, "num_consumers")) {
                to_int(x, p.num_consumers, "Partition.partitions.num_consumers", "int");
            }
        }
    }
    void plist(const JVal& v, PartitionList& pl) {
        if (v.k == JVal::NUL) return;
        if (v.k != JVal::OBJ) {
            if (err.empty()) err = std::string("json: cannot unmarshal ") + kind_name(v) + " into Go value of type main.PartitionList";
            return;
        }
        for (const auto& kv : v.obj) {
            if (fold_eq(kv.first, "version")) {
                to_int(kv.second, pl.version, "PartitionList.version", "int");
            } else if (fold_eq(kv.first, "partitions")) {
                const JVal& a = kv.second;
                if (a.k == JVal::NUL) { pl.partitions.clear(); pl.nil_partitions = true; continue; }
                if (a.k != JVal::ARR) { type_err(a, "PartitionList.partitions", "[]main.Partition"); continue; }
                pl.partitions.clear();
                pl.nil_partitions = false;
                for (const JVal& e : a.arr) {
                    Partition p;
                    partition(e, p);
                    pl.partitions.push_back(std::move(p));
                }
            }
        }
    }
};

// ---- fast path: well-formed documents of the PartitionList shape ----------
// One pass, no DOM: values go straight into the PartitionList.  Whatever it does not
// handle exactly like the DOM parser + Decoder above -- escapes in strings,
// non-integer literals in integer fields, unknown keys, values of unexpected kinds,
// syntax errors, out-of-range numbers -- makes it give up, and the caller runs the
// DOM path, which produces the reference's result or error text.  (The DOM path
// holds a node per number; at c3 size -- 1M partitions with 64-broker lists, ~280 MB
// of JSON -- that is tens of GB.)
struct Fast {
    const char* p;
    const char* e;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    bool lit(char c) {
        ws();
        if (p < e && *p == c) { p++; return true; }
        return false;
    }
    bool null_lit() {
        ws();
        if (e - p >= 4 && memcmp(p, "null", 4) == 0) { p += 4; return true; }
        return false;
    }
    // a string without escapes or control bytes (raw bytes >= 0x80 are copied, as
    // the DOM parser does)
    bool raw_str(const char*& s, size_t& n) {
        ws();
        if (p >= e || *p != '"') return false;
        s = ++p;
        while (p < e && *p != '"' && *p != '\\' && (unsigned char)*p >= 0x20) p++;
        if (p >= e || *p != '"') return false;
        n = (size_t)(p - s);
        p++;
        return true;
    }
    bool key(const char*& s, size_t& n) { return raw_str(s, n) && lit(':'); }
    // an integer literal in int64 range (strtoll's accepted set for JSON integers)
    bool i64(int64_t& v) {
        ws();
        bool neg = false;
        if (p < e && *p == '-') { neg = true; p++; }
        if (p >= e) return false;
        uint64_t m = 0;
        if (*p == '0') p++;
        else if (*p >= '1' && *p <= '9') {
            int nd = 0;
            while (p < e && *p >= '0' && *p <= '9') {
                if (++nd > 19) return false;
                m = m * 10 + (uint64_t)(*p - '0');
                p++;
            }
            if (nd == 19 && m > (neg ? 9223372036854775808ull : 9223372036854775807ull)) return false;
        } else return false;
        if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;   // type error (DOM)
        v = neg ? (int64_t)(0 - m) : (int64_t)m;
        return true;
    }
    // a JSON number (the DOM grammar), converted like strtod; any range issue -> give up
    bool f64(double& v) {
        ws();
        const char* s = p;
        if (p < e && *p == '-') p++;
        if (p >= e) return false;
        if (*p == '0') p++;
        else if (*p >= '1' && *p <= '9') { while (p < e && *p >= '0' && *p <= '9') p++; }
        else return false;
        if (p < e && *p == '.') {
            p++;
            if (p >= e || !(*p >= '0' && *p <= '9')) return false;
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            p++;
            if (p < e && (*p == '+' || *p == '-')) p++;
            if (p >= e || !(*p >= '0' && *p <= '9')) return false;
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        auto r = std::from_chars(s, p, v);
        return r.ec == std::errc() && r.ptr == p && std::isfinite(v);
    }
    std::vector<int64_t> tmp;                          // element staging: one exact allocation per list
    bool ints(Slice& out) {
        if (null_lit()) { out = Slice(); return true; }
        if (!lit('[')) return false;
        tmp.clear();
        if (!lit(']')) {
            for (;;) {
                int64_t x;
                if (!i64(x)) return false;
                tmp.push_back(x);
                if (lit(',')) continue;
                if (lit(']')) break;
                return false;
            }
        }
        out.arr = std::make_shared<std::vector<int64_t>>(tmp.begin(), tmp.end());
        out.len = tmp.size();
        return true;
    }
    static bool is(const char* s, size_t n, const char* name) {
        const size_t m = strlen(name);
        if (n != m) return false;
        for (size_t i = 0; i < n; i++) if (tolower((unsigned char)s[i]) != name[i]) return false;
        return true;
    }
    bool partition(Partition& q) {
        if (null_lit()) return true;
        if (!lit('{')) return false;
        if (lit('}')) return true;
        for (;;) {
            const char* k;
            size_t n;
            if (!key(k, n)) return false;
            bool ok;
            if (is(k, n, "topic")) {
                const char* s;
                size_t m;
                ok = null_lit() || (raw_str(s, m) && (q.topic.assign(s, m), true));
            } else if (is(k, n, "partition")) ok = null_lit() || i64(q.partition);
            else if (is(k, n, "replicas")) ok = ints(q.replicas);
            else if (is(k, n, "weight")) ok = null_lit() || f64(q.weight);
            else if (is(k, n, "num_replicas")) ok = null_lit() || i64(q.num_replicas);
            else if (is(k, n, "brokers")) ok = ints(q.brokers);
            else if (is(k, n, "num_consumers")) ok = null_lit() || i64(q.num_consumers);
            else ok = false;
            if (!ok) return false;
            if (lit(',')) continue;
            if (lit('}')) return true;
            return false;
        }
    }
    // the elements of the "partitions" array after its '[', through the closing ']'
    bool partitions_seq(std::vector<Partition>& v) {
        // (a reserve from the document size: partition objects are >= 16 bytes)
        v.reserve(std::min<size_t>((size_t)(e - p) / 64 + 16, 1u << 26));
        if (lit(']')) return true;
        for (;;) {
            v.emplace_back();
            if (!partition(v.back())) return false;
            if (lit(',')) continue;
            if (lit(']')) return true;
            return false;
        }
    }
    // Large arrays are parsed by several threads, each from a split point: the first
    // '{' after a "}<ws>,<ws>" found near an even share of the bytes.  A split point
    // could lie inside a string, so every chunk but the last must end exactly at the
    // next chunk's start: chunk 0 starts at a true element boundary, and a chunk that
    // starts at one and parses its elements up to the next split point proves that
    // point a boundary too (induction).  Anything else -- a chunk that overruns its
    // end, meets the closing ']' early, or fails -- and the one-thread pass decides.
    bool partitions_body(std::vector<Partition>& v) {
        ws();
        const size_t len = (size_t)(e - p);
        unsigned nt = len < (8u << 20) ? 1u : std::thread::hardware_concurrency();
        if (const char* x = getenv("KB_CODEC_THREADS")) nt = (unsigned)atoi(x);      // tests / benches
        nt = (unsigned)std::max<size_t>(1, std::min<size_t>({(size_t)nt, 16, len / 4096 + 1}));
        if (nt > 1 && partitions_par(v, nt)) return true;
        v.clear();
        return partitions_seq(v);
    }
    bool partitions_par(std::vector<Partition>& v, unsigned nt) {
        const char* a0 = p;
        std::vector<const char*> sp{a0};
        for (unsigned k = 1; k < nt; k++) {
            const char* q = std::max(sp.back() + 1, a0 + (size_t)(e - a0) * k / nt);
            const char* hit = nullptr;
            for (; q < e && !hit; q++) {
                if (*q != '}') continue;
                const char* r = q + 1;
                while (r < e && (*r == ' ' || *r == '\t' || *r == '\n' || *r == '\r')) r++;
                if (r >= e || *r != ',') continue;
                r++;
                while (r < e && (*r == ' ' || *r == '\t' || *r == '\n' || *r == '\r')) r++;
                if (r < e && *r == '{') hit = r;
            }
            if (!hit) break;
            sp.push_back(hit);
        }
        const unsigned nc = (unsigned)sp.size();
        if (nc < 2) return false;
        std::vector<std::vector<Partition>> part(nc);
        std::vector<char> ok(nc, 0);
        const char* tail = nullptr;                   // after the closing ']' (last chunk)
        auto work = [&](unsigned k) {
            Fast g{sp[k], e, {}};
            std::vector<Partition>& out = part[k];
            const bool last = k + 1 == nc;
            out.reserve((size_t)((last ? e : sp[k + 1]) - sp[k]) / 64 + 16);
            for (;;) {
                out.emplace_back();
                if (!g.partition(out.back())) return;
                if (g.lit(',')) {
                    if (last) continue;
                    g.ws();
                    if (g.p == sp[k + 1]) { ok[k] = 1; return; }
                    if (g.p > sp[k + 1]) return;
                    continue;
                }
                if (last && g.lit(']')) { tail = g.p; ok[k] = 1; }
                return;
            }
        };
        std::vector<std::thread> th;
        for (unsigned k = 1; k < nc; k++) th.emplace_back(work, k);
        work(0);
        for (auto& t : th) t.join();
        for (unsigned k = 0; k < nc; k++) if (!ok[k]) return false;
        size_t tot = 0;
        for (const auto& x : part) tot += x.size();
        v.clear();
        v.reserve(tot);
        for (auto& x : part) {
            for (auto& q : x) v.push_back(std::move(q));
            std::vector<Partition>().swap(x);
        }
        p = tail;
        return true;
    }
    bool plist(PartitionList& pl) {
        if (!lit('{')) return false;
        if (lit('}')) return true;
        for (;;) {
            const char* k;
            size_t n;
            if (!key(k, n)) return false;
            if (is(k, n, "version")) {
                if (!null_lit() && !i64(pl.version)) return false;
            } else if (is(k, n, "partitions")) {
                if (null_lit()) { pl.partitions.clear(); pl.nil_partitions = true; }
                else {
                    if (!lit('[')) return false;
                    pl.partitions.clear();
                    pl.nil_partitions = false;
                    if (!partitions_body(pl.partitions)) return false;
                }
            } else return false;
            if (lit(',')) continue;
            if (lit('}')) return true;
            return false;
        }
    }
};

}  // namespace

bool g_codec_dom_only = false;

bool FastDecodePartitionList(const std::string& in, PartitionList* out) {
    PartitionList pl;
    Fast f{in.data(), in.data() + in.size(), {}};
    if (!f.plist(pl)) return false;
    *out = std::move(pl);
    return true;
}

namespace {

// Atoi with the reference's ignored error: value on success, 0 otherwise
int64_t atoi_go(const std::string& s) {
    if (s.empty()) return 0;
    errno = 0;
    char* end = nullptr;
    long long x = strtoll(s.c_str(), &end, 10);
    if (errno || *end) return 0;
    return x;
}

bool take(const std::string& l, size_t& i, const char* lit) {
    size_t n = strlen(lit);
    if (l.compare(i, n, lit) != 0) return false;
    i += n;
    return true;
}
std::string span(const std::string& l, size_t& i, const char* set) {
    size_t st = i;
    while (i < l.size() && strchr(set, l[i]) && l[i]) i++;
    return l.substr(st, i - st);
}

}  // namespace

std::string GetPartitionListFromReader(const std::string& in, bool json,
                                       const std::vector<std::string>& topics, PartitionList* out) {
    PartitionList pl;
    if (json) {
        if (g_codec_dom_only || !FastDecodePartitionList(in, &pl)) {
            pl = PartitionList();
            Parser ps(in);
            ps.ws();
            if (ps.i >= in.size()) return "failed parsing json: EOF";
            JVal v;
            if (!ps.value(v, "looking for beginning of value")) return "failed parsing json: " + ps.err;
            Decoder d;
            d.plist(v, pl);
            if (!d.err.empty()) return "failed parsing json: " + d.err;
        }
        if (pl.version != 1)
            return "wrong partition list version: expected 1, got " + std::to_string((long long)pl.version);
    } else {
        size_t pos = 0;
        while (pos <= in.size()) {
            size_t nl = in.find('\n', pos);
            if (nl == std::string::npos) {
                if (pos == in.size()) break;
                nl = in.size();
            }
            std::string line = in.substr(pos, nl - pos);
            pos = nl + 1;
            if (!line.empty() && line.back() == '\r') line.pop_back();
            if (line.size() > 65536) return "failed reading file: bufio.Scanner: token too long";
            size_t i = 0;
            if (!take(line, i, "\tTopic: ")) continue;
            size_t t0 = i;
            while (i < line.size() && line[i] != '\t') i++;
            std::string topic = line.substr(t0, i - t0);
            if (!take(line, i, "\tPartition: ")) continue;
            std::string part = span(line, i, "0123456789");
            if (!take(line, i, "\tLeader: ")) continue;
            span(line, i, "0123456789");
            if (!take(line, i, "\tReplicas: ")) continue;
            std::string reps = span(line, i, "0123456789,");
            if (!take(line, i, "\tIsr: ")) continue;
            if (!topics.empty()) {
                bool found = false;
                for (const auto& t : topics) found |= t == topic;
                if (!found) continue;
            }
            Partition p;
            p.topic = topic;
            p.partition = atoi_go(part);
            std::vector<int64_t> rs;
            size_t a = 0;
            for (;;) {
                size_t c = reps.find(',', a);
                rs.push_back(atoi_go(reps.substr(a, c == std::string::npos ? std::string::npos : c - a)));
                if (c == std::string::npos) break;
                a = c + 1;
            }
            p.replicas = Slice::of(rs);
            pl.partitions.push_back(std::move(p));
            pl.nil_partitions = false;
        }
    }
    if (pl.partitions.empty()) return "empty partition list";
    *out = std::move(pl);
    return "";
}

// ------------------------------------------------------- JSON output

static void json_string(std::string& o, const std::string& s) {
    static const char* hx = "0123456789abcdef";
    o += '"';
    size_t i = 0;
    while (i < s.size()) {
        unsigned char c = (unsigned char)s[i];
        if (c < 0x80) {
            if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
            else if (c == '\n') o += "\\n";
            else if (c == '\r') o += "\\r";
            else if (c == '\t') o += "\\t";
            else if (c == '\b') o += "\\b";
            else if (c == '\f') o += "\\f";
            else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                o += "\\u00"; o += hx[c >> 4]; o += hx[c & 15];
            } else o += (char)c;
            i++;
            continue;
        }
        // validate one UTF-8 sequence; invalid bytes become � (Go encodeState.string)
        int n = (c >= 0xF0 && c < 0xF5) ? 4 : (c >= 0xE0) ? 3 : (c >= 0xC2 && c < 0xE0) ? 2 : 0;
        bool ok = n > 0 && i + (size_t)n <= s.size();
        uint32_t cp = n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
        for (int k = 1; ok && k < n; k++) {
            unsigned char cc = (unsigned char)s[i + (size_t)k];
            if ((cc & 0xC0) != 0x80) ok = false;
            cp = (cp << 6) | (cc & 0x3F);
        }
        if (ok && ((n == 3 && (cp < 0x800 || (cp >= 0xD800 && cp < 0xE000))) || (n == 4 && (cp < 0x10000 || cp > 0x10FFFF)))) ok = false;
        if (!ok) { o += "\\ufffd"; i++; continue; }
        if (cp == 0x2028 || cp == 0x2029) { o += cp == 0x2028 ? "\\u2028" : "\\u2029"; i += (size_t)n; continue; }
        o.append(s, i, (size_t)n);
        i += (size_t)n;
    }
    o += '"';
}

static void json_int(std::string& o, int64_t v) {
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, v);
    o.append(b, r.ptr);
}

static void json_ints(std::string& o, const Slice& s) {
    if (s.nil()) { o += "null"; return; }
    o += '[';
    for (size_t i = 0; i < s.len; i++) {
        if (i) o += ',';
        json_int(o, s.at(i));
    }
    o += ']';
}

static void encode_partition(std::string& o, const Partition& p) {
    o += "{\"topic\":";
    json_string(o, p.topic);
    o += ",\"partition\":";
    json_int(o, p.partition);
    o += ",\"replicas\":";
    json_ints(o, p.replicas);
    if (p.weight != 0) { o += ",\"weight\":"; GoFloatAppend(o, p.weight); }
    if (p.num_replicas != 0) { o += ",\"num_replicas\":"; json_int(o, p.num_replicas); }
    if (!p.brokers.nil() && p.brokers.len > 0) { o += ",\"brokers\":"; json_ints(o, p.brokers); }
    if (p.num_consumers != 0) { o += ",\"num_consumers\":"; json_int(o, p.num_consumers); }
    o += '}';
}

static size_t encode_estimate(const PartitionList& pl, size_t a, size_t b) {
    size_t est = 0;
    for (size_t i = a; i < b; i++) {
        const Partition& p = pl.partitions[i];
        est += 96 + p.topic.size() + 8 * (p.replicas.len + p.brokers.len);
    }
    return est;
}

// Large lists are encoded in contiguous slices by several threads (the bytes do
// not depend on the split: every partition's text is independent of the others)
std::string EncodePartitionList(PartitionList& pl) {
    pl.version = 1;                                           // codecs.go:86
    std::string o = "{\"version\":1,\"partitions\":";
    if (pl.nil_partitions && pl.partitions.empty()) { o += "null}\n"; return o; }
    const size_t n = pl.partitions.size();
    unsigned nt = n < 65536 ? 1u : std::thread::hardware_concurrency();
    if (const char* v = getenv("KB_CODEC_THREADS")) nt = (unsigned)atoi(v);     // tests / benches
    nt = (unsigned)std::max<size_t>(1, std::min<size_t>({(size_t)nt, 16, n}));
    std::vector<std::string> part(nt);
    auto work = [&](unsigned t) {
        const size_t a = n * t / nt, b = n * (t + 1) / nt;
        std::string& s = part[t];
        s.reserve(encode_estimate(pl, a, b));
        for (size_t i = a; i < b; i++) {
            if (i) s += ',';
            encode_partition(s, pl.partitions[i]);
        }
    };
    if (nt == 1) work(0);
    else {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; t++) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
    }
    size_t tot = o.size() + 3;
    for (const auto& s : part) tot += s.size();
    o.reserve(tot);
    o += '[';
    for (auto& s : part) { o += s; std::string().swap(s); }
    o += "]}\n";
    return o;
}

PartitionList FilterPartitionList(const PartitionList& pl) {
    PartitionList out;
    out.version = pl.version;
    std::set<std::pair<std::string, int64_t>> seen;
    for (const Partition& p : pl.partitions) {
        if (seen.insert({p.topic, p.partition}).second) {
            out.partitions.push_back(p);
            out.nil_partitions = false;
        }
    }
    return out;
}

}  // namespace kbh
