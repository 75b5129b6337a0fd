// bm_json.hpp -- the JSON pieces the C++ host side needs to speak the
// reference's wire formats byte for byte: Go encoding/json's string encoder
// (HTML escaping, \ufffd for invalid UTF-8, utf8.DecodeRuneInString's rules)
// and a strict reader of one flat object (integers range-checked, strings
// unescaped, unknown fields skipped as Go ignores them).  Used by
// btcminer.hpp (bitcoin.Message) and lsp.hpp (lsp.Message).
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>

namespace bmjson {

class DecodeError : public std::runtime_error {
    using std::runtime_error::runtime_error;
};

// One rune of s at i, as Go's utf8.DecodeRuneInString: (rune, size), with
// (0xFFFD, 1) for any invalid or overlong sequence, surrogate or > U+10FFFF.
inline std::pair<uint32_t, size_t> decode_rune(std::string_view s, size_t i) {
    const auto b = [&](size_t k) { return (uint8_t)s[i + k]; };
    const size_t n = s.size() - i;
    const uint8_t c0 = b(0);
    if (c0 < 0x80) return {c0, 1};
    const auto cont = [&](size_t k) { return k < n && (b(k) & 0xC0) == 0x80; };
    if (c0 >= 0xC2 && c0 <= 0xDF && cont(1)) return {((c0 & 0x1Fu) << 6) | (b(1) & 0x3Fu), 2};
    if (c0 >= 0xE0 && c0 <= 0xEF && cont(1) && cont(2)) {
        const uint32_t r = ((c0 & 0x0Fu) << 12) | ((b(1) & 0x3Fu) << 6) | (b(2) & 0x3Fu);
        if (r >= 0x800 && !(r >= 0xD800 && r <= 0xDFFF)) return {r, 3};
    }
    if (c0 >= 0xF0 && c0 <= 0xF4 && cont(1) && cont(2) && cont(3)) {
        const uint32_t r =
            ((c0 & 0x07u) << 18) | ((b(1) & 0x3Fu) << 12) | ((b(2) & 0x3Fu) << 6) | (b(3) & 0x3Fu);
        if (r >= 0x10000 && r <= 0x10FFFF) return {r, 4};
    }
    return {0xFFFD, 1};
}

inline void put_utf8(std::string& out, uint32_t r) {
    if (r < 0x80) {
        out += (char)r;
    } else if (r < 0x800) {
        out += (char)(0xC0 | (r >> 6));
        out += (char)(0x80 | (r & 0x3F));
    } else if (r < 0x10000) {
        out += (char)(0xE0 | (r >> 12));
        out += (char)(0x80 | ((r >> 6) & 0x3F));
        out += (char)(0x80 | (r & 0x3F));
    } else {
        out += (char)(0xF0 | (r >> 18));
        out += (char)(0x80 | ((r >> 12) & 0x3F));
        out += (char)(0x80 | ((r >> 6) & 0x3F));
        out += (char)(0x80 | (r & 0x3F));
    }
}

// encoding/json's string encoder with HTML escaping (json.Marshal's default).
inline std::string go_json_string(std::string_view s) {
    static const char* hex = "0123456789abcdef";
    std::string out = "\"";
    for (size_t i = 0; i < s.size();) {
        const auto [r, size] = decode_rune(s, i);
        if (r == 0xFFFD && size == 1) {
            out += "\\ufffd";  // an invalid byte: Go writes this escape (encoding/json)
        } else if (r == '"' || r == '\\') {
            out += '\\';
            out += (char)r;
        } else if (r == '\n') {
            out += "\\n";
        } else if (r == '\r') {
            out += "\\r";
        } else if (r == '\t') {
            out += "\\t";
        } else if (r < 0x20 || r == '<' || r == '>' || r == '&') {
            out += "\\u00";
            out += hex[r >> 4];
            out += hex[r & 15];
        } else if (r == 0x2028 || r == 0x2029) {
            out += r == 0x2028 ? "\\u2028" : "\\u2029";
        } else {
            out.append(s.substr(i, size));
        }
        i += size;
    }
    out += '"';
    return out;
}

// A strict reader of one flat JSON object (a message's shape).  `what` names
// the message kind in DecodeError texts.
class Reader {
   public:
    explicit Reader(std::string_view s, const char* what = "json") : s_(s), what_(what) {}

    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
    }
    bool eat(char c) {
        ws();
        if (i_ < s_.size() && s_[i_] == c) {
            ++i_;
            return true;
        }
        return false;
    }
    void expect(char c) {
        if (!eat(c)) fail(std::string("expected '") + c + "'");
    }
    bool at_end() {
        ws();
        return i_ == s_.size();
    }
    [[noreturn]] void fail(const std::string& why) const {
        throw DecodeError(std::string(what_) + ": " + why + " at byte " + std::to_string(i_));
    }
    char peek() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        return s_[i_];
    }
    bool literal(std::string_view w) {
        ws();
        if (s_.substr(i_, w.size()) == w) {
            i_ += w.size();
            return true;
        }
        return false;
    }

    std::string string() {
        expect('"');
        std::string out;
        while (true) {
            if (i_ >= s_.size()) fail("unterminated string");
            const uint8_t c = (uint8_t)s_[i_];
            if (c == '"') {
                ++i_;
                return out;
            }
            if (c < 0x20) fail("control character in string");
            if (c == '\\') {
                if (++i_ >= s_.size()) fail("bad escape");
                const char e = s_[i_++];
                switch (e) {
                    case '"': out += '"'; break;
                    case '\\': out += '\\'; break;
                    case '/': out += '/'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 't': out += '\t'; break;
                    case 'u': {
                        uint32_t r = hex4();
                        if (r >= 0xD800 && r <= 0xDBFF && s_.substr(i_, 2) == "\\u") {
                            const size_t save = i_;
                            i_ += 2;
                            const uint32_t lo = hex4();
                            if (lo >= 0xDC00 && lo <= 0xDFFF)
                                r = 0x10000 + ((r - 0xD800) << 10) + (lo - 0xDC00);
                            else
                                i_ = save;
                        }
                        if (r >= 0xD800 && r <= 0xDFFF) r = 0xFFFD;  // a lone surrogate
                        put_utf8(out, r);
                        break;
                    }
                    default: fail("bad escape");
                }
                continue;
            }
            // an invalid raw byte becomes U+FFFD, one per byte, as Go's
            // json.Unmarshal does ("invalid UTF-8 ... replaced by the Unicode
            // replacement character"; utf8.DecodeRune's width-1 RuneError)
            const auto [r, size] = decode_rune(s_, i_);
            if (r == 0xFFFD && size == 1) {
                put_utf8(out, 0xFFFD);
                i_ += 1;
                continue;
            }
            out.append(s_.substr(i_, size));
            i_ += size;
        }
    }

    // An integer literal (no fraction, no exponent) in [lo, hi]; returns
    // false for null.  Booleans, strings, floats and objects are errors.
    bool integer(__int128 lo, __int128 hi, __int128* v) {
        if (literal("null")) return false;
        ws();
        const size_t start = i_;
        bool neg = false;
        if (i_ < s_.size() && s_[i_] == '-') {
            neg = true;
            ++i_;
        }
        if (i_ >= s_.size() || s_[i_] < '0' || s_[i_] > '9') fail("expected an integer");
        if (s_[i_] == '0' && i_ + 1 < s_.size() && s_[i_ + 1] >= '0' && s_[i_ + 1] <= '9') fail("leading zero");
        __int128 x = 0;
        while (i_ < s_.size() && s_[i_] >= '0' && s_[i_] <= '9') {
            x = x * 10 + (s_[i_++] - '0');
            if (x > ((__int128)1 << 65)) fail("integer out of range");
        }
        if (i_ < s_.size() && (s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E')) {
            i_ = start;
            fail("not an integer");
        }
        if (neg) x = -x;
        if (x < lo || x > hi) fail("integer out of range");
        *v = x;
        return true;
    }

    void skip_value() {  // an unknown field's value (Go ignores unknown fields)
        const char c = peek();
        if (c == '"') {
            string();
        } else if (c == '{' || c == '[') {
            const char open = c, close = c == '{' ? '}' : ']';
            expect(open);
            if (eat(close)) return;
            do {
                if (open == '{') {
                    string();
                    expect(':');
                }
                skip_value();
            } while (eat(','));
            expect(close);
        } else if (literal("true") || literal("false") || literal("null")) {
        } else {
            ws();
            const size_t start = i_;
            while (i_ < s_.size() && std::strchr("+-0123456789.eE", s_[i_])) ++i_;
            if (i_ == start) fail("bad value");
        }
    }

   private:
    uint32_t hex4() {
        if (i_ + 4 > s_.size()) fail("bad \\u escape");
        uint32_t r = 0;
        for (int k = 0; k < 4; ++k) {
            const char h = s_[i_++];
            r <<= 4;
            if (h >= '0' && h <= '9') r |= (uint32_t)(h - '0');
            else if (h >= 'a' && h <= 'f') r |= (uint32_t)(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F') r |= (uint32_t)(h - 'A' + 10);
            else fail("bad \\u escape");
        }
        return r;
    }
    std::string_view s_;
    const char* what_;
    size_t i_ = 0;
};


}  // namespace bmjson
