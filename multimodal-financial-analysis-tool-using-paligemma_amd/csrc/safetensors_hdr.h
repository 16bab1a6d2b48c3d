#pragma once
// safetensors_hdr.h -- host-side reader of the safetensors container (the format of the HF
// PaliGemma checkpoints that utils.py:19-44 loads through safe_open / accelerate):
//   [u64 little-endian N][N bytes of JSON header][data]
// header: {"__metadata__": {str: str}, "<tensor>": {"dtype": "BF16", "shape": [..],
//          "data_offsets": [begin, end]}, ...}, offsets relative to the data region.
// Only what the format uses is parsed (objects, strings, integer arrays); anything else in the
// header is skipped structurally.  The file is memory-mapped, so tensor bytes are read straight
// from the page cache into the upload.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace pgmi {

struct StEntry {
    std::string name, dtype;
    std::vector<int64_t> shape;
    int64_t begin = 0, end = 0;
};

struct StFile {
    int fd = -1;
    const uint8_t* map = nullptr;
    size_t size = 0;
    size_t data0 = 0;  // byte offset of the data region
    std::vector<StEntry> entries;
    std::string error;

    ~StFile() {
        if (map) munmap(const_cast<uint8_t*>(map), size);
        if (fd >= 0) close(fd);
    }
};

class StJson {
  public:
    StJson(const char* p, size_t n) : p_(p), e_(p + n) {}
    bool ok() const { return ok_; }

    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
    }
    bool eat(char c) {
        ws();
        if (p_ < e_ && *p_ == c) {
            ++p_;
            return true;
        }
        return false;
    }
    bool peek(char c) {
        ws();
        return p_ < e_ && *p_ == c;
    }
    std::string str() {
        std::string s;
        if (!eat('"')) return fail_s();
        while (p_ < e_ && *p_ != '"') {
            if (*p_ == '\\') {
                if (++p_ >= e_) return fail_s();
                const char c = *p_;
                if (c == 'u') {  // \uXXXX: kept verbatim (tensor names are ASCII)
                    if (e_ - p_ < 5) return fail_s();
                    s.append("\\u").append(p_ + 1, 4);
                    p_ += 5;
                    continue;
                }
                s.push_back(c == 'n' ? '\n' : c == 't' ? '\t' : c == 'r' ? '\r' : c == 'b' ? '\b' : c == 'f' ? '\f' : c);
                ++p_;
                continue;
            }
            s.push_back(*p_++);
        }
        if (!eat('"')) return fail_s();
        return s;
    }
    bool integer(int64_t& v) {
        ws();
        bool neg = false;
        if (p_ < e_ && *p_ == '-') {
            neg = true;
            ++p_;
        }
        if (p_ >= e_ || *p_ < '0' || *p_ > '9') return fail_b();
        int64_t x = 0;
        while (p_ < e_ && *p_ >= '0' && *p_ <= '9') {
            if (x > (INT64_MAX - 9) / 10) return fail_b();
            x = x * 10 + (*p_++ - '0');
        }
        v = neg ? -x : x;
        return true;
    }
    bool int_array(std::vector<int64_t>& out) {
        if (!eat('[')) return fail_b();
        if (eat(']')) return true;
        do {
            int64_t v;
            if (!integer(v)) return false;
            out.push_back(v);
        } while (eat(','));
        return eat(']') || fail_b();
    }
    // skip any value
    bool skip() {
        ws();
        if (p_ >= e_) return fail_b();
        const char c = *p_;
        if (c == '"') {
            str();
            return ok_;
        }
        if (c == '{' || c == '[') {
            const char close = c == '{' ? '}' : ']';
            ++p_;
            if (eat(close)) return true;
            do {
                if (c == '{') {
                    str();
                    if (!eat(':')) return fail_b();
                }
                if (!skip()) return false;
            } while (eat(','));
            return eat(close) || fail_b();
        }
        while (p_ < e_ && *p_ != ',' && *p_ != '}' && *p_ != ']') ++p_;  // number / literal
        return true;
    }

  private:
    std::string fail_s() {
        ok_ = false;
        p_ = e_;
        return {};
    }
    bool fail_b() {
        ok_ = false;
        p_ = e_;
        return false;
    }
    const char* p_;
    const char* e_;
    bool ok_ = true;
};

// open + map + parse; false with f.error set on any malformed input
inline bool st_open(const char* path, StFile& f) {
    f.fd = open(path, O_RDONLY);
    if (f.fd < 0) {
        f.error = std::string("cannot open ") + path;
        return false;
    }
    struct stat sb;
    if (fstat(f.fd, &sb) != 0 || sb.st_size < 8) {
        f.error = std::string("not a safetensors file (too short): ") + path;
        return false;
    }
    f.size = (size_t)sb.st_size;
    void* m = mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, f.fd, 0);
    if (m == MAP_FAILED) {
        f.error = std::string("mmap failed: ") + path;
        return false;
    }
    f.map = reinterpret_cast<const uint8_t*>(m);
    uint64_t n = 0;
    for (int i = 0; i < 8; ++i) n |= (uint64_t)f.map[i] << (8 * i);
    if (n == 0 || n > f.size - 8) {
        f.error = "bad safetensors header length";
        return false;
    }
    f.data0 = 8 + (size_t)n;
    StJson j(reinterpret_cast<const char*>(f.map + 8), (size_t)n);
    if (!j.eat('{')) {
        f.error = "safetensors header is not a JSON object";
        return false;
    }
    if (!j.eat('}')) {
        do {
            const std::string key = j.str();
            if (!j.ok() || !j.eat(':')) break;
            if (key == "__metadata__") {
                if (!j.skip()) break;
                continue;
            }
            StEntry e;
            e.name = key;
            bool have_off = false;
            if (!j.eat('{')) break;
            if (!j.eat('}')) {
                do {
                    const std::string k = j.str();
                    if (!j.ok() || !j.eat(':')) break;
                    if (k == "dtype") {
                        e.dtype = j.str();
                    } else if (k == "shape") {
                        if (!j.int_array(e.shape)) break;
                    } else if (k == "data_offsets") {
                        std::vector<int64_t> o;
                        if (!j.int_array(o) || o.size() != 2) {
                            f.error = "bad data_offsets for " + key;
                            return false;
                        }
                        e.begin = o[0];
                        e.end = o[1];
                        have_off = true;
                    } else if (!j.skip()) {
                        break;
                    }
                } while (j.eat(','));
                if (!j.ok() || !j.eat('}')) break;
            }
            if (!have_off || e.dtype.empty() || e.begin < 0 || e.end < e.begin ||
                (size_t)e.end > f.size - f.data0) {
                f.error = "bad or out-of-range entry " + key;
                return false;
            }
            f.entries.push_back(std::move(e));
        } while (j.eat(','));
        if (!j.ok() || !j.eat('}')) {
            f.error = "malformed safetensors header";
            return false;
        }
    }
    return true;
}

inline int st_elem_bytes(const std::string& dt) {
    if (dt == "BF16" || dt == "F16") return 2;
    if (dt == "F32") return 4;
    return 0;
}

}  // namespace pgmi
