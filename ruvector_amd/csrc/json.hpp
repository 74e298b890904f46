// json.hpp — minimal JSON DOM reader/writer for the RuvectorLayer serde format
// (crates/ruvector-gnn/src/layer.rs:13-17, 50-55, 85-93, 214-227, 314-333;
// ndarray arrays serialise as {"v":1,"dim":[...],"data":[...]}).
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace rvx {
namespace json {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;

    const Value* get(const std::string& k) const {
        for (auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct Parser {
    const char* p;
    const char* end;
    std::string err;

    void ws() {
        while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool fail(const char* m) {
        if (err.empty()) err = m;
        return false;
    }
    bool lit(const char* s) {
        size_t n = strlen(s);
        if ((size_t)(end - p) < n || strncmp(p, s, n) != 0) return fail("bad literal");
        p += n;
        return true;
    }
    bool parse_string(std::string& out) {
        if (p >= end || *p != '"') return fail("expected string");
        ++p;
        while (p < end && *p != '"') {
            if (*p == '\\') {
                ++p;
                if (p >= end) return fail("bad escape");
                char c = *p++;
                switch (c) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (end - p < 4) return fail("bad \\u escape");
                        unsigned cp = (unsigned)strtoul(std::string(p, 4).c_str(), nullptr, 16);
                        p += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += c;
                }
            } else {
                out += *p++;
            }
        }
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    bool parse(Value& v, int depth = 0) {
        if (depth > 64) return fail("nesting too deep");
        ws();
        if (p >= end) return fail("unexpected end");
        char c = *p;
        if (c == '{') {
            ++p;
            v.kind = Value::Object;
            ws();
            if (p < end && *p == '}') { ++p; return true; }
            while (true) {
                ws();
                std::string k;
                if (!parse_string(k)) return false;
                ws();
                if (p >= end || *p != ':') return fail("expected ':'");
                ++p;
                Value child;
                if (!parse(child, depth + 1)) return false;
                v.obj.emplace_back(std::move(k), std::move(child));
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == '}') { ++p; return true; }
                return fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++p;
            v.kind = Value::Array;
            ws();
            if (p < end && *p == ']') { ++p; return true; }
            while (true) {
                Value child;
                if (!parse(child, depth + 1)) return false;
                v.arr.push_back(std::move(child));
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == ']') { ++p; return true; }
                return fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.kind = Value::String; return parse_string(v.str); }
        if (c == 't') { v.kind = Value::Bool; v.b = true; return lit("true"); }
        if (c == 'f') { v.kind = Value::Bool; v.b = false; return lit("false"); }
        if (c == 'n') { v.kind = Value::Null; return lit("null"); }
        // number
        char* e = nullptr;
        std::string tmp;
        const char* s = p;
        while (p < end && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E')) ++p;
        tmp.assign(s, p);
        if (tmp.empty()) return fail("unexpected character");
        v.kind = Value::Number;
        v.num = strtod(tmp.c_str(), &e);
        if (!e || *e != 0) return fail("bad number");
        return true;
    }
};

inline bool parse(const std::string& text, Value& out, std::string& err) {
    Parser ps{text.data(), text.data() + text.size(), {}};
    if (!ps.parse(out)) { err = ps.err; return false; }
    ps.ws();
    if (ps.p != ps.end) { err = "trailing characters"; return false; }
    return true;
}

// f32 -> shortest-ish decimal that round-trips through strtof.
inline void put_f32(std::string& s, float f) {
    if (std::isnan(f) || std::isinf(f)) { s += "null"; return; }
    char buf[32];
    for (int prec = 6; prec <= 9; ++prec) {
        snprintf(buf, sizeof buf, "%.*g", prec, (double)f);
        if (strtof(buf, nullptr) == f) break;
    }
    s += buf;
    // serde_json always prints a decimal point or exponent for floats
    if (!strpbrk(buf, ".eE")) s += ".0";
}

}  // namespace json
}  // namespace rvx
