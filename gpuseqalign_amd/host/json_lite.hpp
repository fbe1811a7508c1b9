// json_lite.hpp -- the small JSON subset the reference's input files use (subst.json,
// algorithm-parameter files): objects (key order kept), arrays, integers, strings, bools,
// null, with // and /* */ comments allowed (the reference parses them with comments enabled,
// src/io.hpp:33).  Header-only; errors throw JsonError with a line:column position.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace gsa_host {

struct JsonError : std::runtime_error
{
    using std::runtime_error::runtime_error;
};

struct Json
{
    enum class Kind { Null, Bool, Int, String, Array, Object };
    Kind kind = Kind::Null;
    bool b = false;
    int64_t i = 0;
    std::string s;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;  // insertion order

    bool is_object() const { return kind == Kind::Object; }
    bool is_array() const { return kind == Kind::Array; }
    bool is_int() const { return kind == Kind::Int; }
    const Json* find(const std::string& key) const
    {
        for (auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

class JsonParser
{
public:
    explicit JsonParser(const std::string& text) : t_(text) {}

    Json parse()
    {
        Json v = value();
        ws();
        if (p_ != t_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& t_;
    size_t p_ = 0;

    [[noreturn]] void fail(const char* what) const
    {
        size_t line = 1, col = 1;
        for (size_t k = 0; k < p_ && k < t_.size(); ++k)
        {
            if (t_[k] == '\n') { ++line; col = 1; }
            else ++col;
        }
        throw JsonError(std::to_string(line) + ":" + std::to_string(col) + ": " + what);
    }

    void ws()
    {
        for (;;)
        {
            while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t' || t_[p_] == '\n' || t_[p_] == '\r')) ++p_;
            if (p_ + 1 < t_.size() && t_[p_] == '/' && t_[p_ + 1] == '/')
            {
                while (p_ < t_.size() && t_[p_] != '\n') ++p_;
                continue;
            }
            if (p_ + 1 < t_.size() && t_[p_] == '/' && t_[p_ + 1] == '*')
            {
                size_t e = t_.find("*/", p_ + 2);
                if (e == std::string::npos) fail("unterminated comment");
                p_ = e + 2;
                continue;
            }
            return;
        }
    }

    bool lit(const char* w)
    {
        size_t n = std::char_traits<char>::length(w);
        if (t_.compare(p_, n, w) == 0)
        {
            p_ += n;
            return true;
        }
        return false;
    }

    std::string str()
    {
        if (t_[p_] != '"') fail("expected string");
        ++p_;
        std::string out;
        while (p_ < t_.size() && t_[p_] != '"')
        {
            char c = t_[p_++];
            if (c == '\\')
            {
                if (p_ >= t_.size()) fail("bad escape");
                char e = t_[p_++];
                switch (e)
                {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'u':
                    if (p_ + 4 > t_.size()) fail("bad \\u escape");
                    out += (char)std::stoi(t_.substr(p_, 4), nullptr, 16);  // ASCII subset only
                    p_ += 4;
                    break;
                default: out += e;
                }
            }
            else
                out += c;
        }
        if (p_ >= t_.size()) fail("unterminated string");
        ++p_;
        return out;
    }

    Json value()
    {
        ws();
        if (p_ >= t_.size()) fail("unexpected end of input");
        Json v;
        char c = t_[p_];
        if (c == '{')
        {
            v.kind = Json::Kind::Object;
            ++p_;
            ws();
            if (p_ < t_.size() && t_[p_] == '}') { ++p_; return v; }
            for (;;)
            {
                ws();
                std::string k = str();
                ws();
                if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
                ++p_;
                v.obj.emplace_back(std::move(k), value());
                ws();
                if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
                if (p_ < t_.size() && t_[p_] == '}') { ++p_; return v; }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[')
        {
            v.kind = Json::Kind::Array;
            ++p_;
            ws();
            if (p_ < t_.size() && t_[p_] == ']') { ++p_; return v; }
            for (;;)
            {
                v.arr.push_back(value());
                ws();
                if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
                if (p_ < t_.size() && t_[p_] == ']') { ++p_; return v; }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"')
        {
            v.kind = Json::Kind::String;
            v.s = str();
            return v;
        }
        if (lit("true")) { v.kind = Json::Kind::Bool; v.b = true; return v; }
        if (lit("false")) { v.kind = Json::Kind::Bool; v.b = false; return v; }
        if (lit("null")) return v;
        if (c == '-' || (c >= '0' && c <= '9'))
        {
            size_t q = p_;
            if (t_[q] == '-') ++q;
            while (q < t_.size() && t_[q] >= '0' && t_[q] <= '9') ++q;
            if (q < t_.size() && (t_[q] == '.' || t_[q] == 'e' || t_[q] == 'E')) fail("only integer numbers are supported");
            v.kind = Json::Kind::Int;
            v.i = std::stoll(t_.substr(p_, q - p_));
            p_ = q;
            return v;
        }
        fail("unexpected character");
    }
};

inline Json parse_json(const std::string& text) { return JsonParser(text).parse(); }

}  // namespace gsa_host
