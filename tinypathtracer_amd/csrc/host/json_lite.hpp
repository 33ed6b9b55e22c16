// json_lite.hpp -- minimal JSON DOM for the glTF loader (host only).
#pragma once

#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace tpt {
namespace json {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;   // file order

    bool is_null() const { return kind == Null; }
    bool is_object() const { return kind == Object; }
    bool is_array() const { return kind == Array; }
    bool is_number() const { return kind == Number; }

    const Value* find(const std::string& key) const {
        if (kind != Object) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    double number_or(const std::string& key, double dflt) const {
        const Value* v = find(key);
        return (v && v->kind == Number) ? v->num : dflt;
    }
    // Integer field; a number outside +-2^62 (or NaN) is out of range for any
    // index, offset or count and reads as `bad` (the double -> integer cast
    // would be undefined behaviour there).
    long long int_or(const std::string& key, long long dflt, long long bad = -1) const {
        const Value* v = find(key);
        if (!v || v->kind != Number) return dflt;
        if (!(v->num >= -4.6e18 && v->num <= 4.6e18)) return bad;
        return (long long)v->num;
    }
    std::string string_or(const std::string& key, const std::string& dflt) const {
        const Value* v = find(key);
        return (v && v->kind == String) ? v->str : dflt;
    }
    size_t size() const { return kind == Array ? arr.size() : (kind == Object ? obj.size() : 0); }
    const Value& operator[](size_t i) const {
        if (kind != Array || i >= arr.size()) throw std::runtime_error("json: index out of range");
        return arr[i];
    }
};

class Parser {
public:
    explicit Parser(const std::string& text) : s_(text), i_(0) {}
    Value parse() {
        Value v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_;
    int depth_ = 0;   // open containers; glTF nests a few levels, a hostile file thousands
    static constexpr int kMaxDepth = 128;
    struct Nest {
        Parser& p;
        explicit Nest(Parser& q) : p(q) {
            if (++p.depth_ > kMaxDepth) p.fail("nesting too deep");
        }
        ~Nest() { --p.depth_; }
    };

    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i_));
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
    }
    bool lit(const char* w) {
        size_t n = 0;
        while (w[n]) ++n;
        if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
        return false;
    }
    Value value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        Value v;
        if (c == '{') {
            Nest nest(*this);
            v.kind = Value::Object;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
            for (;;) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') fail("expected key");
                std::string k = string_body();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
                ++i_;
                v.obj.emplace_back(std::move(k), value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
                if (i_ < s_.size() && s_[i_] == '}') { ++i_; break; }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            Nest nest(*this);
            v.kind = Value::Array;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
                if (i_ < s_.size() && s_[i_] == ']') { ++i_; break; }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            v.kind = Value::String;
            v.str = string_body();
        } else if (lit("true")) {
            v.kind = Value::Bool; v.b = true;
        } else if (lit("false")) {
            v.kind = Value::Bool; v.b = false;
        } else if (lit("null")) {
            v.kind = Value::Null;
        } else {
            const char* start = s_.c_str() + i_;
            char* end = nullptr;
            double d = std::strtod(start, &end);       // correctly rounded decimal -> double
            if (end == start) fail("bad value");
            i_ += (size_t)(end - start);
            v.kind = Value::Number;
            v.num = d;
        }
        return v;
    }
    static void put_utf8(std::string& o, unsigned cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        }
    }
    unsigned hex4() {
        if (i_ + 4 > s_.size()) fail("bad \\u escape");
        unsigned v = (unsigned)std::stoul(s_.substr(i_, 4), nullptr, 16);
        i_ += 4;
        return v;
    }
    std::string string_body() {
        ++i_;   // opening quote
        std::string o;
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c != '\\') { o += c; continue; }
            if (i_ >= s_.size()) fail("bad escape");
            char e = s_[i_++];
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
                    unsigned cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                        i_ += 2;
                        unsigned lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(o, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        if (i_ >= s_.size()) fail("unterminated string");
        ++i_;
        return o;
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace json
}  // namespace tpt
