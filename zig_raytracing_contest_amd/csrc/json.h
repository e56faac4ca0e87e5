// json.h -- minimal JSON DOM for glTF and config.json (RFC 8259 subset:
// objects, arrays, strings with escapes incl. \uXXXX, numbers, true/false/null).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace zrt {
namespace json {

struct Value {
    enum Type { Null, Bool, Number, String, Array, Object } type = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;

    const Value* get(const char* key) const {
        if (type != Object) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    double number(const char* key, double dflt) const {
        const Value* v = get(key);
        return (v && v->type == Number) ? v->num : dflt;
    }
    int64_t integer(const char* key, int64_t dflt) const {
        const Value* v = get(key);
        return (v && v->type == Number) ? (int64_t)v->num : dflt;
    }
    std::string string(const char* key, const char* dflt) const {
        const Value* v = get(key);
        return (v && v->type == String) ? v->str : std::string(dflt);
    }
    size_t size() const { return type == Array ? arr.size() : (type == Object ? obj.size() : 0); }
    const Value& operator[](size_t i) const { return arr[i]; }
};

class Parser {
  public:
    Parser(const char* s, size_t n) : p_(s), end_(s + n) {}
    bool parse(Value* out) {
        ws();
        if (!value(out, 0)) return false;
        ws();
        return p_ == end_;
    }

  private:
    const char* p_;
    const char* end_;

    void ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char* w) {
        const size_t n = strlen(w);
        if ((size_t)(end_ - p_) < n || memcmp(p_, w, n) != 0) return false;
        p_ += n;
        return true;
    }
    static void utf8(uint32_t cp, std::string* o) {
        if (cp < 0x80) o->push_back((char)cp);
        else if (cp < 0x800) { o->push_back((char)(0xC0 | (cp >> 6))); o->push_back((char)(0x80 | (cp & 63))); }
        else if (cp < 0x10000) {
            o->push_back((char)(0xE0 | (cp >> 12)));
            o->push_back((char)(0x80 | ((cp >> 6) & 63)));
            o->push_back((char)(0x80 | (cp & 63)));
        } else {
            o->push_back((char)(0xF0 | (cp >> 18)));
            o->push_back((char)(0x80 | ((cp >> 12) & 63)));
            o->push_back((char)(0x80 | ((cp >> 6) & 63)));
            o->push_back((char)(0x80 | (cp & 63)));
        }
    }
    bool hex4(uint32_t* v) {
        if (end_ - p_ < 4) return false;
        *v = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = *p_++;
            *v <<= 4;
            if (c >= '0' && c <= '9') *v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') *v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') *v |= (uint32_t)(c - 'A' + 10);
            else return false;
        }
        return true;
    }
    bool string(std::string* o) {
        if (p_ >= end_ || *p_ != '"') return false;
        ++p_;
        while (p_ < end_ && *p_ != '"') {
            char c = *p_++;
            if ((unsigned char)c < 0x20) return false;
            if (c != '\\') { o->push_back(c); continue; }
            if (p_ >= end_) return false;
            c = *p_++;
            switch (c) {
                case '"': o->push_back('"'); break;
                case '\\': o->push_back('\\'); break;
                case '/': o->push_back('/'); break;
                case 'b': o->push_back('\b'); break;
                case 'f': o->push_back('\f'); break;
                case 'n': o->push_back('\n'); break;
                case 'r': o->push_back('\r'); break;
                case 't': o->push_back('\t'); break;
                case 'u': {
                    uint32_t cp;
                    if (!hex4(&cp)) return false;
                    if (cp >= 0xD800 && cp < 0xDC00) {
                        uint32_t lo;
                        if (!lit("\\u") || !hex4(&lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(cp, o);
                    break;
                }
                default: return false;
            }
        }
        if (p_ >= end_) return false;
        ++p_;
        return true;
    }
    bool number(double* v) {
        const char* s = p_;
        if (p_ < end_ && *p_ == '-') ++p_;
        if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return false;
        while (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                             *p_ == '+' || *p_ == '-'))
            ++p_;
        std::string tmp(s, p_);
        char* e = nullptr;
        *v = strtod(tmp.c_str(), &e);
        return e && *e == 0;
    }
    bool value(Value* v, int depth) {
        if (depth > 256 || p_ >= end_) return false;
        const char c = *p_;
        if (c == '{') {
            ++p_;
            v->type = Value::Object;
            ws();
            if (p_ < end_ && *p_ == '}') { ++p_; return true; }
            for (;;) {
                ws();
                std::string k;
                if (!string(&k)) return false;
                ws();
                if (p_ >= end_ || *p_ != ':') return false;
                ++p_;
                ws();
                v->obj.emplace_back(std::move(k), Value());
                if (!value(&v->obj.back().second, depth + 1)) return false;
                ws();
                if (p_ < end_ && *p_ == ',') { ++p_; continue; }
                if (p_ < end_ && *p_ == '}') { ++p_; return true; }
                return false;
            }
        }
        if (c == '[') {
            ++p_;
            v->type = Value::Array;
            ws();
            if (p_ < end_ && *p_ == ']') { ++p_; return true; }
            for (;;) {
                ws();
                v->arr.emplace_back();
                if (!value(&v->arr.back(), depth + 1)) return false;
                ws();
                if (p_ < end_ && *p_ == ',') { ++p_; continue; }
                if (p_ < end_ && *p_ == ']') { ++p_; return true; }
                return false;
            }
        }
        if (c == '"') { v->type = Value::String; return string(&v->str); }
        if (lit("true")) { v->type = Value::Bool; v->b = true; return true; }
        if (lit("false")) { v->type = Value::Bool; v->b = false; return true; }
        if (lit("null")) { v->type = Value::Null; return true; }
        v->type = Value::Number;
        return number(&v->num);
    }
};

inline bool parse(const char* s, size_t n, Value* out) { return Parser(s, n).parse(out); }

}  // namespace json
}  // namespace zrt
