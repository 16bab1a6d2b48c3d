/*
 * oracle/wgen.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Deterministic synthetic-weight generator shared by the oracle, the golden
 * fixture script and the parity tests.  PaliGemma weights/tokenizer are not
 * available offline (SURVEY.md sec.7 "hard parts" 8), so parity is defined on
 * synthetic weights that every party can regenerate bit-exactly:
 *
 *   key   = splitmix64(seed ^ fnv1a64(state_dict_name))
 *   u_i   = splitmix64(key + i)                     (i = flat element index)
 *   v_i   = ((int)(u_i >> 40) - 2^23) * 2^-23       (uniform in [-1, 1), exact f32)
 *   w_i   = bf16_rne( offset + v_i * scale )        (two f32 ops, NO fma contraction)
 *
 * The product library implements the same recipe on the device
 * (pgmi_fill_synthetic, csrc/synthetic.hip) for the benchmark; the GPU test
 * suite checks the two agree bit-for-bit.
 *
 * Build: gcc -O2 -ffp-contract=off -shared -fPIC wgen.c -o libwgen.so
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

uint64_t wgen_name_hash(const char* name) {
    uint64_t h = 0xCBF29CE484222325ULL;
    for (const unsigned char* p = (const unsigned char*)name; *p; ++p) {
        h ^= *p;
        h *= 0x100000001B3ULL;
    }
    return h;
}

static inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

/* Fill out[0..n) (bf16 bit patterns) for tensor `name`. */
void wgen_fill_bf16(const char* name, uint64_t seed, float scale, float offset,
                    uint16_t* out, int64_t n) {
    const uint64_t key = splitmix64(seed ^ wgen_name_hash(name));
    for (int64_t i = 0; i < n; ++i) {
        uint64_t u = splitmix64(key + (uint64_t)i);
        float v = (float)((int32_t)(u >> 40) - (1 << 23)) * (1.0f / 8388608.0f);
        volatile float t = v * scale; /* keep the two roundings separate */
        float w = offset + t;
        out[i] = f32_to_bf16_rne(w);
    }
}

/* Same values widened to f32 (the bf16 value, exactly). */
void wgen_fill_f32(const char* name, uint64_t seed, float scale, float offset,
                   float* out, int64_t n) {
    const uint64_t key = splitmix64(seed ^ wgen_name_hash(name));
    for (int64_t i = 0; i < n; ++i) {
        uint64_t u = splitmix64(key + (uint64_t)i);
        float v = (float)((int32_t)(u >> 40) - (1 << 23)) * (1.0f / 8388608.0f);
        volatile float t = v * scale;
        float w = offset + t;
        uint32_t b = (uint32_t)f32_to_bf16_rne(w) << 16;
        memcpy(&out[i], &b, 4);
    }
}
