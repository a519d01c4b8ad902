// json_lite.hpp — minimal JSON reader for the SchemaJSON vocabulary
// (schema/schemabuilder_json.go:8-30).  Host-only.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace packos {

struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0;
    std::string str;        // STR: the string; NUM: the literal's text (exact int64 parsing)
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;

    const JVal* get(const std::string& k) const {
        if (kind != OBJ) return nullptr;
        for (auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    bool truthy() const { return kind == BOOL ? b : (kind == NUM ? num != 0 : false); }
};

class JParser {
public:
    explicit JParser(const std::string& s) : s_(s) {}
    JVal parse() {
        JVal v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_ = 0;
    [[noreturn]] void fail(const char* m) {
        throw std::runtime_error(std::string("schema JSON: ") + m + " at offset " + std::to_string(i_));
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) i_++;
    }
    bool lit(const char* w) {
        size_t n = std::char_traits<char>::length(w);
        if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
        return false;
    }
    JVal value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        JVal v;
        if (c == '{') {
            v.kind = JVal::OBJ; i_++; ws();
            if (i_ < s_.size() && s_[i_] == '}') { i_++; return v; }
            for (;;) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') fail("expected key");
                std::string k = string();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
                i_++;
                v.obj.emplace_back(k, value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { i_++; continue; }
                if (i_ < s_.size() && s_[i_] == '}') { i_++; return v; }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = JVal::ARR; i_++; ws();
            if (i_ < s_.size() && s_[i_] == ']') { i_++; return v; }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { i_++; continue; }
                if (i_ < s_.size() && s_[i_] == ']') { i_++; return v; }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.kind = JVal::STR; v.str = string(); return v; }
        if (lit("true")) { v.kind = JVal::BOOL; v.b = true; return v; }
        if (lit("false")) { v.kind = JVal::BOOL; v.b = false; return v; }
        if (lit("null")) { v.kind = JVal::NUL; return v; }
        if (c == '-' || (c >= '0' && c <= '9')) {
            size_t st = i_;
            i_++;
            while (i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '.' || s_[i_] == 'e' ||
                                      s_[i_] == 'E' || s_[i_] == '+' || s_[i_] == '-'))
                i_++;
            v.kind = JVal::NUM;
            v.str = s_.substr(st, i_ - st);
            v.num = std::stod(v.str);
            return v;
        }
        fail("unexpected character");
    }
    static void put_utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        }
    }
    std::string string() {
        std::string o;
        i_++;  // opening quote
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
                    if (i_ + 4 > s_.size()) fail("bad \\u escape");
                    uint32_t cp = (uint32_t)std::stoul(s_.substr(i_, 4), nullptr, 16);
                    i_ += 4;
                    if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                        uint32_t lo = (uint32_t)std::stoul(s_.substr(i_ + 2, 4), nullptr, 16);
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        i_ += 6;
                    }
                    put_utf8(o, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        if (i_ >= s_.size()) fail("unterminated string");
        i_++;
        return o;
    }
};

}  // namespace packos
