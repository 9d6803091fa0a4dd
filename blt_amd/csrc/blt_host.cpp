// Host side of the MI355X BPE merge scan: the C ABI of include/blt_bpe.h.
//
// Owns the merges loader (config_loader.rs:14-46), the config helpers (utils.rs, chunking.rs),
// the strategy handle (BpeStrategy, tokenizer.rs:43-93) with its device tables, the per-pass
// orchestration of the kernels in bpe_kernels.hip, and the multi-GPU chunk sharding that
// replaces the reference's tokio task-per-chunk pipeline (pipeline.rs:56-192).
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/blt_bpe.h"
#include "bpe_kernels.h"

namespace {

thread_local std::string t_err;

int fail(int code, const char* fmt, ...) {
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

}  // namespace

namespace blt_internal {
int set_error(int code, const char* fmt, ...) {
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}
}  // namespace blt_internal

namespace {

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(BLT_E_IO, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// No C++ exception may cross the C ABI: every int-returning entry point runs its body in GUARDED.
#define GUARDED(...)                                                                    \
    try {                                                                               \
        __VA_ARGS__                                                                     \
    } catch (const std::bad_alloc&) {                                                   \
        return fail(BLT_E_NOMEM, "out of host memory");                                 \
    } catch (const std::exception& e_) {                                                \
        return fail(BLT_E_IO, "%s", e_.what());                                         \
    } catch (...) {                                                                     \
        return fail(BLT_E_IO, "unexpected C++ exception");                              \
    }

// ---------------------------------------------------------------------------------------
// Text helpers for the loader: Rust's BufRead::lines() / str::split_whitespace / FromStr.
// ---------------------------------------------------------------------------------------
// Length of the UTF-8 sequence at p (code point in *cp), 0 if malformed.
size_t utf8_seq(const unsigned char* p, size_t n, uint32_t* cp) {
    if (!n) return 0;
    const unsigned c = p[0];
    if (c < 0x80) { *cp = c; return 1; }
    size_t len = (c >= 0xF0 && c <= 0xF4) ? 4 : (c >= 0xE0) && c < 0xF0 ? 3 : (c >= 0xC2 && c < 0xE0) ? 2 : 0;
    if (!len || len > n) return 0;
    uint32_t v = c & (len == 2 ? 0x1F : len == 3 ? 0x0F : 0x07);
    for (size_t i = 1; i < len; ++i) {
        if ((p[i] & 0xC0) != 0x80) return 0;
        v = (v << 6) | (p[i] & 0x3F);
    }
    static const uint32_t kMin[5] = {0, 0, 0x80, 0x800, 0x10000};
    if (v < kMin[len] || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return 0;
    *cp = v;
    return len;
}

bool is_white_space(uint32_t c) {  // Unicode White_Space (char::is_whitespace)
    switch (c) {
        case 0x20: case 0x85: case 0xA0: case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F:
        case 0x3000: return true;
        default: return (c >= 0x09 && c <= 0x0D) || (c >= 0x2000 && c <= 0x200A);
    }
}

// Fields of str::split_whitespace over a valid UTF-8 line.
std::vector<std::string> split_whitespace(const std::string& s) {
    std::vector<std::string> out;
    const auto* p = reinterpret_cast<const unsigned char*>(s.data());
    size_t i = 0, start = 0;
    bool in = false;
    while (i < s.size()) {
        uint32_t cp = 0;
        size_t l = utf8_seq(p + i, s.size() - i, &cp);
        if (!l) l = 1;
        if (is_white_space(cp)) {
            if (in) out.emplace_back(s, start, i - start);
            in = false;
        } else if (!in) {
            in = true;
            start = i;
        }
        i += l;
    }
    if (in) out.emplace_back(s, start);
    return out;
}

// <uN as FromStr>::from_str in radix 10: optional sign handling of core::num for unsigned
// types; per char the digit check comes before the overflow check.  "" on success, else the
// ParseIntError text.
const char* parse_unsigned(const std::string& s, uint64_t limit, uint64_t* out) {
    if (s.empty()) return "cannot parse integer from empty string";
    size_t i = 0;
    if (s[0] == '+' || s[0] == '-') {
        if (s.size() == 1) return "invalid digit found in string";
        if (s[0] == '+') i = 1;
    }
    uint64_t r = 0;
    for (; i < s.size(); ++i) {
        const bool mul_ok = r <= limit / 10;
        if (s[i] < '0' || s[i] > '9') return "invalid digit found in string";
        if (!mul_ok) return "number too large to fit in target type";
        r *= 10;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (r > limit - d) return "number too large to fit in target type";
        r += d;
    }
    *out = r;
    return "";
}

// load_bpe_merges_from_path (config_loader.rs:14-46) into a dense (a, b) -> id table
// (-1 absent).  Returns 0 or a BLT_E_* code with t_err set to the io::Error text.
int load_merges_table(const char* path, std::vector<int32_t>& table) {
    // File::open + read_line (config_loader.rs:15-21): an OS error is "<strerror> (os error N)"
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
        const int e = errno;
        return fail(e == ENOENT ? BLT_E_NOT_FOUND : BLT_E_IO, "%s (os error %d)", strerror(e), e);
    }
    std::string data;
    char buf[1 << 16];
    for (;;) {
        const ssize_t r = ::read(fd, buf, sizeof buf);
        if (r < 0) {
            if (errno == EINTR) continue;
            const int e = errno;   // e.g. EISDIR for a directory
            ::close(fd);
            return fail(BLT_E_IO, "%s (os error %d)", strerror(e), e);
        }
        if (r == 0) break;
        data.append(buf, (size_t)r);
    }
    ::close(fd);
    table.assign(65536, -1);
    uint16_t vocab = 256;  // :18, wraps like the release build (no overflow-checks)
    size_t pos = 0;
    while (pos < data.size()) {
        size_t nl = data.find('\n', pos);
        const bool had_nl = nl != std::string::npos;
        const size_t end = had_nl ? nl : data.size();
        // read_line validates the bytes it appends, newline included
        {
            const auto* p = reinterpret_cast<const unsigned char*>(data.data()) + pos;
            size_t i = 0, len = end - pos + (had_nl ? 1 : 0);
            while (i < len) {
                uint32_t cp;
                size_t l = utf8_seq(p + i, len - i, &cp);
                if (!l) return fail(BLT_E_INVALID_DATA, "stream did not contain valid UTF-8");
                i += l;
            }
        }
        std::string line = data.substr(pos, end - pos);
        if (had_nl && !line.empty() && line.back() == '\r') line.pop_back();  // lines(): "\r\n"
        pos = had_nl ? nl + 1 : end;
        if (line.empty() || line[0] == '#') continue;  // :22
        const std::vector<std::string> parts = split_whitespace(line);
        if (parts.size() != 2)  // :41-43
            return fail(BLT_E_INVALID_DATA,
                        "Invalid merge rule format in line: '%s'. Expected two numbers separated by space.",
                        line.c_str());
        uint64_t b1 = 0, b2 = 0;
        const char* e1 = parse_unsigned(parts[0], 255, &b1);
        if (*e1) return fail(BLT_E_INVALID_DATA, "Failed to parse first byte value: %s in line '%s'", e1, line.c_str());
        const char* e2 = parse_unsigned(parts[1], 255, &b2);
        if (*e2) return fail(BLT_E_INVALID_DATA, "Failed to parse second byte value: %s in line '%s'", e2, line.c_str());
        table[(b1 << 8) | b2] = vocab;  // :39 insert (last wins)
        vocab = (uint16_t)(vocab + 1);   // :40
    }
    return 0;
}

uint64_t total_ram_bytes() {
    FILE* f = fopen("/proc/meminfo", "r");
    if (!f) return 0;
    char key[64];
    unsigned long long kb = 0;
    uint64_t r = 0;
    while (fscanf(f, "%63s %llu kB", key, &kb) == 2) {
        if (strcmp(key, "MemTotal:") == 0) { r = (uint64_t)kb * 1024ull; break; }
    }
    fclose(f);
    return r;
}

}  // namespace

// ===========================================================================================
// Strategy handle
// ===========================================================================================
constexpr int kMaxDevices = 64;

struct DevTables {
    std::once_flag once;
    int status = 0;
    uint16_t* dense = nullptr;      // native u16 values, sentinel where absent (general kernel)
    uint16_t* self_ne = nullptr;    // self-token table, native byte order (byte-pass kernel)
    uint16_t* self_be = nullptr;    // self-token table, output (big-endian) byte order
    uint2* hbuckets = nullptr;      // general map: cuckoo buckets (u16 passes)
};

struct blt_bpe {
    size_t n_entries = 0;
    bool single_pass = true;
    uint32_t sentinel = 0;                 // > 0xFFFF: every byte pair is a merge
    std::vector<uint16_t> dense;           // 65536, swizzled (blt::dense_index)
    // Self-token tables of the byte-pass kernel: entry (a, b) = merged token, or a itself when
    // (a, b) is no merge.  byte_mode, the kernel's merge test (launch_scan_bytes): 0 every byte-pair
    // merge value is >= 256 (every merges file: ids 256 + line), so "merge" is the entry's high
    // byte; 1 the entry differs from a; 2 as 1, with merges valued their own first byte a stored as
    // (mark << 8) | a, mark a high byte no merge value has; -1 none applies (the generic byte pass).
    // allmerge: every byte pair is a merge (the test is skipped).
    int byte_mode = 0;
    bool allmerge = false;
    uint32_t mark = 0;
    // A general map whose keys are all byte pairs: its first pass reports whether it made a token
    // below 256 (the only key components), and is the fixpoint when it made none.
    bool live_first = false;
    // A byte-pair key (a, a): a run of that byte merges pair after pair, so the fused first two
    // passes could find no restart in a wave range's halo; such maps keep the two-kernel chain.
    bool byte_self_pair = false;
    // General map: the longest merge chain (chain_depth; 0 = unbounded): the passes it needs are
    // known up front, so they are enqueued without reading the device's pass count.
    uint32_t chain_depth = 0;
    std::vector<uint16_t> self_ne, self_be;
    // General map (not single_pass): 2-choice cuckoo table of one-slot buckets for the u16 passes
    // (blt::bucket_of), words [key, val]; key = BE(a) | BE(b) << 16, val = BE(value) | 1 << 31
    // | 1 << 30 when the value is a component of some key.
    std::vector<uint32_t> hwords;
    uint32_t hmul1 = 0, hmul2 = 0, hshift = 0;
    bool hone = false;                     // one-probe table (hmul2 == hmul1)
    DevTables dev[kMaxDevices];
    // Sticky device-error word in pinned, mapped host memory: any kernel of this handle that flags
    // an error (look-back timeout, output range, prefix invariant) stores 1 here, and every later
    // call on the handle fails with BLT_E_IO until blt_bpe_clear_error.  An async encode cannot
    // report its own failure, but the caller's next call does.
    // Published once under sticky_once with a release store; read with acquire loads, so a thread
    // that checks it before its own first sticky_word() never races the allocating thread.
    std::once_flag sticky_once;
    std::atomic<uint32_t*> sticky{nullptr};
    // Pinned host words of the sparse passes' reads (SparseHost), one per concurrent encode: taken
    // from this free list and returned after the run, freed by blt_bpe_destroy.
    mutable std::mutex sp_mu;
    mutable std::vector<void*> sp_free;
};

namespace {

// 2-choice cuckoo placement of the general map (u16 passes): one-slot buckets [key, value],
// load at most one half, dot2 hashes of the key's u16 halves (blt::bucket_of); new multipliers
// (and then twice the buckets) until every key has a place.  The key of (a, b) is the pair's
// u16 words as stored, BE(a) | BE(b) << 16; empty buckets hold a key that is not in the map.
// Values carry bit 30 when the merged token is a component of some key (is_comp): the u16 scan
// kernel stops the passes after one that made no such token.
bool build_buckets(const std::unordered_map<uint32_t, uint16_t>& map, const std::vector<uint8_t>& is_comp, blt_bpe* h) {
    auto be = [](uint32_t v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); };
    std::vector<uint32_t> keys, vals;
    keys.reserve(map.size());
    vals.reserve(map.size());
    for (const auto& kv : map) {
        keys.push_back(be(kv.first >> 16) | (be(kv.first & 0xFFFFu) << 16));
        vals.push_back(be(kv.second) | 0x80000000u | (is_comp[kv.second] ? 0x40000000u : 0u));
    }
    std::unordered_set<uint32_t> keyset(keys.begin(), keys.end());
    uint32_t empty = 0xFFFFFFFFu;
    while (keyset.count(empty)) --empty;
    uint32_t log2nb = 2;
    while ((1ull << log2nb) < 2 * map.size()) ++log2nb;
    uint64_t seed = 0x9E3779B97F4A7C15ull;
    auto next_mul = [&seed]() {
        seed = seed * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)(seed >> 32) | 0x00010001u;   // two odd 16-bit multipliers
    };
    // Small maps first try a one-probe table (every key in its own bucket of one hash), up to
    // 4096 buckets (32 KiB of LDS): the u16 scan kernel then reads one bucket per lookup.
    for (uint32_t l2 = log2nb; keys.size() <= 512 && l2 <= 12; ++l2) {
        const uint32_t nb = 1u << l2, shift = 32 - l2;
        for (int attempt = 0; attempt < 64; ++attempt) {
            const uint32_t m1 = next_mul();
            std::vector<uint32_t> key(nb, empty), val(nb, 0);
            bool ok = true;
            for (size_t i = 0; i < keys.size() && ok; ++i) {
                const uint32_t b = blt::bucket_of(keys[i], m1, shift);
                ok = key[b] == empty;
                key[b] = keys[i];
                val[b] = vals[i];
            }
            if (!ok) continue;
            h->hwords.assign(2ull * nb, 0);
            for (uint32_t i = 0; i < nb; ++i) {
                h->hwords[2 * i] = key[i];
                h->hwords[2 * i + 1] = val[i];
            }
            h->hmul1 = h->hmul2 = m1;
            h->hshift = shift;
            h->hone = true;
            return true;
        }
    }
    for (; log2nb <= 25; ++log2nb) {
        const uint32_t nb = 1u << log2nb, shift = 32 - log2nb;
        for (int attempt = 0; attempt < 32; ++attempt) {
            const uint32_t m1 = next_mul(), m2 = next_mul();
            std::vector<uint32_t> key(nb, empty), val(nb, 0);
            bool ok = true;
            for (size_t i = 0; i < keys.size() && ok; ++i) {
                uint32_t k = keys[i], v = vals[i];
                uint32_t b = blt::bucket_of(k, m1, shift);
                bool placed = false;
                for (int kick = 0; kick < 512 && !placed; ++kick) {
                    const uint32_t b1 = blt::bucket_of(k, m1, shift), b2 = blt::bucket_of(k, m2, shift);
                    if (key[b1] == empty) { key[b1] = k; val[b1] = v; placed = true; break; }
                    if (key[b2] == empty) { key[b2] = k; val[b2] = v; placed = true; break; }
                    // evict the occupant of b (alternating between the key's two buckets) and carry
                    // it to its other bucket
                    b = (kick & 1) ? b2 : b1;
                    std::swap(k, key[b]);
                    std::swap(v, val[b]);
                }
                ok = placed;
            }
            if (!ok) continue;
            h->hwords.assign(2ull * nb, 0);
            for (uint32_t i = 0; i < nb; ++i) {
                h->hwords[2 * i] = key[i];
                h->hwords[2 * i + 1] = val[i];
            }
            h->hmul1 = m1;
            h->hmul2 = m2;
            h->hshift = shift;
            return true;
        }
    }
    return false;
}

// Longest merge chain of a general map: D(v) = 1 + max over keys (x, y) -> v of max(D(x), D(y)), and
// D = 0 for a token no key produces.  A merge in u16 pass p involves a token pass p - 1 produced (a
// pair of two older tokens was looked up in pass p - 1 and rejected), so it ends a chain of p + 1
// merges: no pass after the max D-th merges anything.  0 when some value can be made from itself
// (a cycle: the chain is unbounded, e.g. (97, 98) -> 97 on "abbb...").
uint32_t chain_depth(const std::unordered_map<uint32_t, uint16_t>& map) {
    std::unordered_map<uint32_t, std::vector<uint32_t>> prod;   // value -> keys that make it
    for (const auto& kv : map) prod[kv.second].push_back(kv.first);
    std::vector<uint32_t> depth(65536, 0);
    std::vector<uint8_t> state(65536, 0);   // 0 unseen, 1 on the DFS stack, 2 done
    struct Frame { uint32_t v; size_t i; uint32_t best; };
    uint32_t maxd = 0;
    for (const auto& pv : prod) {
        if (state[pv.first]) continue;
        std::vector<Frame> st{{pv.first, 0, 0}};
        state[pv.first] = 1;
        while (!st.empty()) {
            Frame& f = st.back();
            const std::vector<uint32_t>& ks = prod[f.v];
            if (f.i < 2 * ks.size()) {
                const uint32_t key = ks[f.i / 2];
                const uint32_t c = (f.i & 1) ? (key & 0xFFFFu) : (key >> 16);
                ++f.i;
                if (!prod.count(c)) continue;                  // not a value: depth 0
                if (state[c] == 1) return 0;                   // a cycle
                if (state[c] == 2) { f.best = std::max(f.best, depth[c]); continue; }
                state[c] = 1;
                st.push_back({c, 0, 0});
                continue;
            }
            depth[f.v] = f.best + 1;
            state[f.v] = 2;
            maxd = std::max(maxd, depth[f.v]);
            const uint32_t d = depth[f.v];
            st.pop_back();
            if (!st.empty()) st.back().best = std::max(st.back().best, d);
        }
    }
    return maxd;
}

int build_handle(const std::vector<uint32_t>& keys, const std::vector<uint16_t>& vals, blt_bpe** out) {
    std::unique_ptr<blt_bpe> h(new (std::nothrow) blt_bpe());
    if (!h) return fail(BLT_E_NOMEM, "out of host memory");
    // Final map: later duplicates overwrite (HashMap collect).
    std::unordered_map<uint32_t, uint16_t> map;
    map.reserve(keys.size() * 2 + 1);
    for (size_t i = 0; i < keys.size(); ++i) map[keys[i]] = vals[i];
    h->n_entries = map.size();

    // One pass is the fixpoint when no value is a key component: after pass 1 two adjacent
    // raw bytes were adjacent in the input and already rejected, and a merged token can match
    // no key.
    std::vector<uint8_t> is_value(65536, 0), is_comp(65536, 0);
    for (const auto& kv : map) {
        is_value[kv.second] = 1;
        is_comp[kv.first >> 16] = 1;
        is_comp[kv.first & 0xFFFF] = 1;
    }
    for (int t = 0; t < 65536 && h->single_pass; ++t)
        if (is_value[t] && is_comp[t]) h->single_pass = false;
    if (!h->single_pass) h->chain_depth = chain_depth(map);

    // Dense byte-pair table for pass 1: value, or a sentinel no byte-pair key maps to.
    std::vector<uint8_t> used(65536, 0);
    size_t byte_pairs = 0;
    for (const auto& kv : map)
        if ((kv.first >> 16) < 256 && (kv.first & 0xFFFF) < 256) { used[kv.second] = 1; ++byte_pairs; }
    if (byte_pairs == 65536) {
        h->sentinel = 0x10000u;
    } else {
        uint32_t s = 0xFFFF;
        while (used[s]) --s;  // at most 65535 values are used, so one is free
        h->sentinel = s;
    }
    h->dense.assign(65536, (uint16_t)(h->sentinel & 0xFFFF));
    for (const auto& kv : map) {
        const uint32_t a = kv.first >> 16, b = kv.first & 0xFFFF;
        if (a < 256 && b < 256) h->dense[blt::dense_index(a, b)] = kv.second;
    }
    auto bswap = [](uint32_t v) { return (uint16_t)(((v & 0xFF) << 8) | ((v >> 8) & 0xFF)); };
    bool hi_merge = true, self_valued = false, byte_keys = true;
    std::vector<uint8_t> hi_used(256, 0);   // high bytes of byte-pair merge values
    for (const auto& kv : map) {
        const uint32_t a = kv.first >> 16, b = kv.first & 0xFFFF;
        if (a < 256 && b < 256) {
            if (a == b) h->byte_self_pair = true;
            if (kv.second == a) self_valued = true;
            if (kv.second < 256) hi_merge = false;
            hi_used[kv.second >> 8] = 1;
        } else {
            byte_keys = false;
        }
    }
    h->allmerge = byte_pairs == 65536;
    if (hi_merge) {
        h->byte_mode = 0;
    } else if (!self_valued || h->allmerge) {
        h->byte_mode = 1;
    } else {
        h->byte_mode = -1;
        for (uint32_t m = 1; m < 256 && h->byte_mode < 0; ++m)
            if (!hi_used[m]) { h->byte_mode = 2; h->mark = m; }
    }
    h->live_first = !h->single_pass && byte_keys && h->byte_mode > 0;
    h->self_ne.assign(blt::kSelfEntries, 0);
    for (uint32_t a = 0; a < 256; ++a)
        for (uint32_t b = 0; b < 256; ++b) h->self_ne[blt::self_index(a, b)] = (uint16_t)a;
    for (const auto& kv : map) {
        const uint32_t a = kv.first >> 16, b = kv.first & 0xFFFF;
        if (a < 256 && b < 256)
            h->self_ne[blt::self_index(a, b)] = (h->byte_mode == 2 && kv.second == a) ? (uint16_t)((h->mark << 8) | a)
                                                                                     : kv.second;
    }
    h->self_be.resize(blt::kSelfEntries);
    for (uint32_t i = 0; i < blt::kSelfEntries; ++i) h->self_be[i] = bswap(h->self_ne[i]);
    if (!h->single_pass && !build_buckets(map, is_comp, h.get())) return fail(BLT_E_NOMEM, "cannot place the merge map in a hash table");
    *out = h.release();
    return 0;
}

int current_device(int* dev) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1) return fail(BLT_E_NODEV, "no HIP device available");
    HIP_TRY(hipGetDevice(dev));
    if (*dev < 0 || *dev >= kMaxDevices) return fail(BLT_E_NODEV, "device index %d out of range", *dev);
    return 0;
}

// BLT_CLI_TIMING: a setup step's end (seconds since the first such stamp), on stderr
void detail_stamp(const char* what) {
    static const bool on = getenv("BLT_CLI_TIMING") != nullptr;
    if (!on) return;
    static timespec t0 = [] { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t; }();
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    fprintf(stderr, "blt timing: detail: %s %.4f s\n", what,
            (double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec));
}

int device_tables(const blt_bpe* hc, int dev, DevTables** out, hipStream_t via = nullptr) {
    blt_bpe* h = const_cast<blt_bpe*>(hc);
    DevTables& t = h->dev[dev];
    // Upload on a private stream (or the caller's idle stream `via`) and wait for it: the kernels
    // run on non-blocking streams, which do not order behind null-stream copies.  (Each stream the
    // process creates costs the CLI's start-up ~10 ms: BLT_CLI_TIMING's detail stamps.)
    std::call_once(t.once, [&]() {
        // one allocation and one copy (separate ones cost the CLI's start-up: profiles/r05_cli_phases.json)
        auto up256 = [](size_t x) { return (x + 255) & ~size_t(255); };
        const size_t b_dense = 65536 * sizeof(uint16_t), b_self = blt::kSelfEntries * sizeof(uint16_t);
        const size_t b_hash = h->hwords.size() * sizeof(uint32_t);
        const size_t o_ne = up256(b_dense), o_be = o_ne + up256(b_self), o_hash = o_be + up256(b_self);
        const size_t total = o_hash + up256(b_hash);
        std::vector<uint8_t> blob(total, 0);
        memcpy(blob.data(), h->dense.data(), b_dense);
        memcpy(blob.data() + o_ne, h->self_ne.data(), b_self);
        memcpy(blob.data() + o_be, h->self_be.data(), b_self);
        if (b_hash) memcpy(blob.data() + o_hash, h->hwords.data(), b_hash);
        hipStream_t us = via;
        uint8_t* base = nullptr;
        detail_stamp("tables: blob built");
        bool ok = us || hipStreamCreateWithFlags(&us, hipStreamNonBlocking) == hipSuccess;
        detail_stamp("tables: stream created");
        ok = ok && hipMalloc(&base, total) == hipSuccess;
        detail_stamp("tables: allocated");
        ok = ok && hipMemcpyAsync(base, blob.data(), total, hipMemcpyHostToDevice, us) == hipSuccess;
        detail_stamp("tables: copy issued");
        if (base) {   // (blt_bpe_destroy frees `dense`, the allocation's start)
            t.dense = reinterpret_cast<uint16_t*>(base);
            t.self_ne = reinterpret_cast<uint16_t*>(base + o_ne);
            t.self_be = reinterpret_cast<uint16_t*>(base + o_be);
            if (b_hash) t.hbuckets = reinterpret_cast<uint2*>(base + o_hash);
        }
        ok = ok && hipStreamSynchronize(us) == hipSuccess;
        detail_stamp("tables: copied");
        if (us && us != via) (void)hipStreamDestroy(us);
        detail_stamp("tables: stream destroyed");
        if (!ok) t.status = BLT_E_IO;
    });
    if (t.status) return fail(t.status, "uploading merge tables to device %d failed", dev);
    *out = &t;
    return 0;
}

// The handle's sticky error word (pinned, mapped, portable: one host word every device can
// store to), allocated on first device use.  nullptr if the allocation failed.
uint32_t* sticky_word(const blt_bpe* hc) {
    blt_bpe* h = const_cast<blt_bpe*>(hc);
    std::call_once(h->sticky_once, [h] {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) == hipSuccess) {
            memset(p, 0, 64);
            h->sticky.store(static_cast<uint32_t*>(p), std::memory_order_release);
        }
    });
    return h->sticky.load(std::memory_order_acquire);
}

// BLT_E_IO if a kernel of this handle flagged a device error since the last blt_bpe_clear_error.
int sticky_check(const blt_bpe* h) {
    const uint32_t* w = h->sticky.load(std::memory_order_acquire);
    if (w && __atomic_load_n(w, __ATOMIC_ACQUIRE))
        return fail(BLT_E_IO,
                    "a previous merge scan on this handle flagged a device error (look-back timeout, output range "
                    "or prefix invariant); its output is invalid (blt_bpe_clear_error resets the handle)");
    return 0;
}

// Test hook: per-tile look-back records (blt_debug_set_tile_record).
uint64_t* g_debug_tiles = nullptr;
// Test hook (blt_debug_set_inject): blt::kInject* bits, counts the kernels break on purpose.
std::atomic<uint32_t> g_inject{0};
// Test hook: n_gpus contexts even where they share a device (blt_debug_set_shared_contexts).
std::atomic<int> g_shared_contexts{0};
// Passes 1 and 2 of eligible general maps in one kernel (blt_debug_set_fused(0): the two-kernel
// chain, for A/B runs and tests).
std::atomic<int> g_fused{1};
// Test hooks (blt_debug_set_u16_chain): bit 0 chained scan passes build the next pass's chunk map,
// bit 1 the host extends the scan kernel's chunk bound from the offsets it reads.
std::atomic<int> g_u16_chain{3};
// Test hook (blt_debug_set_fused_only): a synchronous general-map encode that ran the fused kernel
// returns right after it (its tokens in d_out, its count; chunk offsets not copied out).
std::atomic<int> g_fused_only{0};
constexpr uint32_t kEncodeNoFused = 1u << 31;   // internal encode_device flag: the two-kernel chain
// Test hook: u16 passes the calling thread's last synchronous general-map encode ran before the
// chain stopped (blt_debug_last_u16_passes).
thread_local uint32_t t_last_u16_passes = 0;
// Test hook: u16 passes the calling thread's last general-map encode enqueued on the scan kernel
// (blt_debug_last_scan_passes).
thread_local uint32_t t_last_scan_passes = 0;
// Test hook: how the calling thread's last synchronous general-map encode ran passes 1 and 2:
// 0 two kernels, 1 fused, 2 fused and fell back (blt_debug_last_fused).
thread_local uint32_t t_last_fused = 0;

// ---- workspace layout -------------------------------------------------------------------
inline uint64_t up16(uint64_t x) { return (x + 15) & ~15ull; }
inline uint64_t up256(uint64_t x) { return (x + 255) & ~255ull; }

struct WsLayout {
    uint64_t ntiles, nchunks;
    uint64_t ctl, status, status2, total, off_a, off_b, cmap, cmap_stride, gstat, bytes, zero_bytes;
    // sparse passes of a cyclic map (run_sparse): bitmaps of n bits, seed and merge lists of
    // sp_cap entries, compaction tile words, counters; sp_cap 0 when the map cannot use them
    uint64_t sp_holes, sp_bits0, sp_bits1, sp_bits2, sp_seeds0, sp_seeds1, sp_merges, sp_tileo, sp_status, sp_ctr, sp_ntiles,
        sp_slices;
    uint32_t sp_cap;
};
// Longest chain enqueued without reading the pass count (deeper chains run in host-checked batches).
constexpr uint32_t kMaxBoundedPasses = 64;
inline bool chain_bounded(const blt_bpe* h) { return h->chain_depth && h->chain_depth <= kMaxBoundedPasses + 1; }
// Sparse passes per run_sparse call (one counter pair each, zeroed once; a longer tail goes back to
// the full passes).  Counter words: [0] overflow flag, [1] unused, [2 + p] pass p's seeds,
// [2 + kSparseMaxPasses + 1 + p] pass p's merges.
constexpr uint32_t kSparseMaxPasses = 250;
constexpr uint32_t kSparseCtrWords = 2 + 2 * (kSparseMaxPasses + 1);
// Chain block of a general map (right after pass 1's status words): u64 pass totals [2], u32 done
// word, u32 fused-fail word, u64 final total, u32 finish-gate word, pad.
constexpr uint64_t kChainBlock = 48;

// Workspace: control block and look-back status words (zeroed before each pass), then for a
// general map the pass totals and done flag, two chunk-offset arrays (the passes alternate) and
// the chunk map of the u16 scan kernel (one word per kTokRange tokens).  The u16 passes run in
// place in the caller's output.
WsLayout ws_layout(const blt_bpe* h, uint64_t n, uint64_t cs) {
    const bool single_pass = h->single_pass;
    WsLayout L{};
    const uint64_t tile = single_pass ? std::min<uint64_t>(blt::kTilePos, blt::kTilePosBytes)
                                      : std::min<uint64_t>(blt::kTilePosTok, blt::kTilePosBytes);
    L.ntiles = (n + tile - 1) / tile;
    L.nchunks = n ? (n + cs - 1) / cs : 0;
    L.ctl = 0;
    L.status = blt::kCtlBytes;
    L.zero_bytes = up16(blt::kCtlBytes + 8 * L.ntiles);
    L.total = L.zero_bytes;   // the chain block (kChainBlock bytes, right after pass 1's status
                              // words: encode_device zeroes both at once)
    L.off_a = L.total + kChainBlock;
    L.off_b = L.off_a + up16(8 * (L.nchunks + 1));
    // three chunk maps: u16 scan pass k reads map k % 3, builds k + 1's and zeroes k + 2's (each on
    // cache lines of its own: one is zeroed while the next is marked)
    L.cmap = up256(L.off_b + up16(8 * (L.nchunks + 1)));
    L.cmap_stride = up256(8 * ((n + blt::kTokRange - 1) / blt::kTokRange));
    L.gstat = L.cmap + 3 * L.cmap_stride;   // finish: a status word per group
    // the second set of look-back status words of chained u16 passes (U16Run; the first is pass 1's)
    L.status2 = up256(L.gstat + up16(8 * L.nchunks));
    L.bytes = single_pass ? L.cmap : L.status2 + up16(8 * L.ntiles);
    if (!single_pass && !chain_bounded(h) && n < (1ull << 32)) {
        const uint64_t bm = up16(4 * ((n + 31) / 32));
        const uint64_t cap = n / 16 + 4096;
        const uint64_t sptiles = (n + blt::kSparseTile - 1) / blt::kSparseTile;
        L.sp_cap = (uint32_t)cap;
        L.sp_ntiles = sptiles;
        L.sp_holes = up16(L.bytes);
        L.sp_bits0 = L.sp_holes + bm;
        L.sp_bits1 = L.sp_bits0 + bm;
        L.sp_bits2 = L.sp_bits1 + bm;
        L.sp_seeds0 = L.sp_bits2 + bm;
        L.sp_seeds1 = L.sp_seeds0 + up16(4 * cap);
        L.sp_merges = L.sp_seeds1 + up16(4 * cap);
        L.sp_tileo = L.sp_merges + up16(12 * cap);
        L.sp_status = L.sp_tileo + up16(4 * ((sptiles + 15) & ~15ull) + 16);
        L.sp_ctr = L.sp_status + up16(8 * sptiles);
        // + the gate's sample, then the list slices' counts: seeds (two, alternating by pass), merges
        L.sp_slices = L.sp_ctr + up16(4ull * kSparseCtrWords) + 4ull * blt::kSparseSampleBlocks;
        L.bytes = L.sp_slices + 3ull * 4ull * blt::kSparseSlices;
    }
    return L;
}

int read_u64(const void* dptr, uint64_t* v, hipStream_t s) {
    HIP_TRY(hipMemcpyAsync(v, dptr, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
}

int ctl_error(const uint32_t* ctl) {
    if (ctl[1])
        return fail(BLT_E_IO,
                    "merge-scan device check failed (flags 0x%x: 1 look-back timeout, 2 output range, 4 prefix "
                    "invariant, 8 workgroup wait timeout, 16 chunk map, 32 workspace not zeroed for this size "
                    "(BLT_ENCODE_WORKSPACE_ZEROED past the last reset), 64 finish-kernel count invariant; first "
                    "at tile %u sub-tile %u, O=%llu, value=%llu, C=%u)",
                    ctl[1], ctl[2] ? ctl[2] - 1 : 0, ctl[3], (unsigned long long)ctl[4] | ((unsigned long long)ctl[5] << 32),
                    (unsigned long long)ctl[6] | ((unsigned long long)ctl[7] << 32), ctl[8]);
    return 0;
}

int check_ctl(uint8_t* ws, hipStream_t s) {
    uint32_t ctl[16] = {0};
    HIP_TRY(hipMemcpyAsync(ctl, ws, sizeof ctl, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return ctl_error(ctl);
}

// Enqueues one merge pass over n positions.
// u16 passes of a general map: the token count comes from the device and is written there.
struct Chain {
    const uint64_t* n_in = nullptr;   // count written by the previous pass
    uint64_t* n_out = nullptr;        // this pass's count
    uint32_t* done = nullptr;         // set to its pass_id by the last pass that can merge anything
    uint32_t pass_id = 0;             // 1, 2, ...
    bool next_scan = false;           // the next pass runs on the scan kernel too (it builds its chunk map)
};

// What the previous launch of a chain left for the next u16 pass (round 6).  Chained u16 passes
// (scan or merge kernel) alternate two sets of look-back status words and ticket words; each pass
// zeroes the other set for the pass after it, so only the first pass of a run needs the chunk-map
// kernel (scan) or a memset (merge) to zero its own.  Any other kernel in between (the finish or
// sparse kernels) resets it.
struct U16Run {
    bool map_ready = false;   // the previous pass was a scan pass that built this pass's chunk map
    bool st_ready = false;    // the previous pass zeroed set `par`'s status words and ticket
    uint32_t par = 0;         // the set this pass uses: 0 pass 1's status words and ctl[0], 1 the others
    void reset() { map_ready = st_ready = false; }
};

// tok_scan: a u16 pass on the scan kernel (every chunk holds >= kTokRange tokens).  run (u16 passes
// of a chain): see U16Run, updated for the next pass.
int run_pass(const blt_bpe* h, const DevTables* t, int dev, hipStream_t s, uint8_t* ws, const WsLayout& L,
             const void* in, bool in_u16, uint64_t n, uint64_t cs, const uint64_t* cstart, void* out, bool be,
             uint64_t out_cap, uint64_t* chunk_off, bool ws_zeroed = false, const Chain* chain = nullptr,
             bool tok_scan = false, U16Run* run = nullptr) {
    const bool columnar = !in_u16 && cs >= blt::kMinChunkBytes && h->byte_mode >= 0 && be;   // byte-pass fast kernel
    const uint64_t tile = columnar ? blt::kTilePosBytes
                                   : in_u16 ? (tok_scan ? blt::kTilePosTok : blt::kTilePosU16) : blt::kTilePos;
    const uint64_t ntiles = (n + tile - 1) / tile;
    if (ntiles > 0xFFFFFFFFull) return fail(BLT_E_INVALID_INPUT, "input too large");
    if (!(g_u16_chain.load(std::memory_order_relaxed) & 1)) run = nullptr;
    const bool chained = in_u16 && chain && run;
    // (the u16 scan's chunk-map kernel zeroes the control block and status words itself, and a
    // chained pass finds them zeroed by the pass before it)
    const bool merge_ready = chained && !tok_scan && run->st_ready;
    if (!ws_zeroed && !(in_u16 && tok_scan) && !merge_ready) {
        HIP_TRY(hipMemsetAsync(ws, 0, up16(blt::kCtlBytes + 8 * ntiles), s));
        if (chained) run->par = 0;   // (the memset zeroed set 0: the control block and pass 1's words)
    }
    blt::PassParams p{};
    p.in = in;
    p.n = n;
    p.cs = cs;
    p.cstart = cstart;
    p.nchunks = L.nchunks;
    p.out = out;
    p.out_cap = out_cap;
    p.chunk_off = chunk_off;
    p.status = reinterpret_cast<uint64_t*>(ws + L.status);
    p.ctl = reinterpret_cast<uint32_t*>(ws + L.ctl);
    p.total = chain ? chain->n_out : reinterpret_cast<uint64_t*>(ws + L.total);
    if (chain) {
        p.n_dev = chain->n_in;
        p.done = chain->done;
        p.pass_id = chain->pass_id;
    }
    p.ntiles = (uint32_t)ntiles;
    p.sentinel = h->sentinel;
    p.dense = columnar ? (be ? t->self_be : t->self_ne) : t->dense;
    p.hbuckets = t->hbuckets;
    p.hmul1 = h->hmul1;
    p.hmul2 = h->hmul2;
    p.hshift = h->hshift;
    p.hbytes = (uint32_t)(h->hwords.size() * sizeof(uint32_t));
    p.hone = h->hone ? 1u : 0u;
    p.cs_magic = cs ? ~0ull / cs : 0;
    if (cs && cs % blt::kTilePosBytes == 0 && cs / blt::kTilePosBytes < (1ull << 31)) {
        p.cs_tiles = (uint32_t)(cs / blt::kTilePosBytes);
        p.cs_tiles_magic = p.cs_tiles > 1 ? (uint32_t)(0xFFFFFFFFull / p.cs_tiles) : 0u;
    }
    p.allm = h->allmerge ? 1u : 0u;
    p.mark = h->mark | (h->mark << 16);
    p.debug = g_debug_tiles;
    p.inject = g_inject.load(std::memory_order_relaxed);
    p.sticky = h->sticky.load(std::memory_order_acquire);
    const bool scan16 = in_u16 && tok_scan;
    const bool ready = scan16 && chained && run->map_ready;
    auto map = [&](uint32_t i) { return reinterpret_cast<uint64_t*>(ws + L.cmap + (uint64_t)(i % 3u) * L.cmap_stride); };
    const uint32_t r = chain ? chain->pass_id % 3u : 0u;
    if (scan16) p.cmap = map(r);
    if (chained) {
        // this pass's set of status words and ticket, zeroed by the pass before it (or by the
        // chunk-map kernel or the memset); the other set zeroed here for the next pass
        const bool alt = run->par != 0;
        p.status = reinterpret_cast<uint64_t*>(ws + (alt ? L.status2 : L.status));
        p.status_zero = reinterpret_cast<uint64_t*>(ws + (alt ? L.status : L.status2));
        p.tick = alt ? blt::kCtlTickAlt : 0u;
        if (scan16 && chain->next_scan) {   // the next pass's chunk map, built here
            p.cmap_next = map(r + 1u);
            p.cmap_zero = map(r + 2u);
        }
        run->par ^= 1u;
        run->st_ready = true;
        run->map_ready = scan16 && chain->next_scan;
    }
    p.ws_check = (ws_zeroed && !in_u16 && !chain) ? 1u : 0u;   // the caller's BLT_ENCODE_WORKSPACE_ZEROED
    if (columnar) HIP_TRY(blt::launch_scan_bytes(p, h->byte_mode, (chain && h->live_first) ? 1 : 0, dev, s));
    else if (scan16) {
        HIP_TRY(blt::launch_scan_tokens(p, ready ? 1 : 0, dev, s));
        ++t_last_scan_passes;
    }
    else HIP_TRY(blt::launch_merge_pass(p, in_u16 ? 1 : 0, be ? 1 : 0, dev, s));
    return 0;
}

// Passes 1 and 2 of a general map in one launch (blt::launch_scan_fused): bytes d_in to the second
// pass's tokens in d_out, its total, chunk offsets and done word as u16 pass 1's.
int run_fused(const blt_bpe* h, const DevTables* t, int dev, hipStream_t s, uint8_t* ws, const WsLayout& L,
              const uint8_t* d_in, uint64_t n, uint64_t cs, uint8_t* d_out, uint64_t* chunk_off, uint64_t* total,
              uint32_t* done, uint32_t* fused_fail) {
    const uint64_t ntiles = (n + blt::kTilePosTok - 1) / blt::kTilePosTok;
    if (ntiles > 0xFFFFFFFFull) return fail(BLT_E_INVALID_INPUT, "input too large");
    blt::PassParams p{};
    p.in = d_in;
    p.n = n;
    p.cs = cs;
    p.nchunks = L.nchunks;
    p.out = d_out;
    p.out_cap = 2 * n;
    p.chunk_off = chunk_off;
    p.status = reinterpret_cast<uint64_t*>(ws + L.status);
    p.ctl = reinterpret_cast<uint32_t*>(ws + L.ctl);
    p.total = total;
    p.done = done;
    p.pass_id = 1;
    p.ntiles = (uint32_t)ntiles;
    p.hbuckets = t->hbuckets;
    p.hmul1 = h->hmul1;
    p.hmul2 = h->hmul2;
    p.hshift = h->hshift;
    p.hbytes = (uint32_t)(h->hwords.size() * sizeof(uint32_t));
    p.hone = h->hone ? 1u : 0u;
    p.cs_magic = ~0ull / cs;
    p.debug = g_debug_tiles;
    p.inject = g_inject.load(std::memory_order_relaxed);
    p.sticky = h->sticky.load(std::memory_order_acquire);
    p.fused_fail = fused_fail;
    HIP_TRY(blt::launch_scan_fused(p, dev, s));
    return 0;
}

// The rest of a general map's chain from u16 pass k on, per group of chunks in LDS (blt::launch_finish):
// tokens in place in d_out, chunk starts from the previous pass's offsets, this pass's offsets and
// total as pass k's.  Enqueued once per encode, at the first pass whose input chunks may fit in LDS
// (a pass at least halves a chunk's tokens: they hold >= cs >> k entering u16 pass k); when a group
// does not fit after all, the gate leaves it to the ordinary pass k enqueued right behind it.
int run_finish(const blt_bpe* h, const DevTables* t, int dev, hipStream_t s, uint8_t* ws, const WsLayout& L,
               uint8_t* d_out, uint32_t k, const uint64_t* off_in, uint64_t* off_out, uint64_t* total, uint32_t* done) {
    blt::PassParams p{};
    p.in = d_out;
    p.out = d_out;
    p.cstart = off_in;
    p.nchunks = L.nchunks;
    p.chunk_off = off_out;
    p.total = total;
    p.done = done;
    p.pass_id = k;
    p.status = reinterpret_cast<uint64_t*>(ws + L.gstat);
    p.ctl = reinterpret_cast<uint32_t*>(ws + L.ctl);
    p.hbuckets = t->hbuckets;
    p.hmul1 = h->hmul1;
    p.hmul2 = h->hmul2;
    p.hshift = h->hshift;
    p.hbytes = (uint32_t)(h->hwords.size() * sizeof(uint32_t));
    p.hone = h->hone ? 1u : 0u;
    p.sticky = h->sticky.load(std::memory_order_acquire);
    p.fin_gate = reinterpret_cast<uint32_t*>(ws + L.total + 32);
    p.debug = g_debug_tiles;
    p.inject = g_inject.load(std::memory_order_relaxed);
    HIP_TRY(blt::launch_finish(p, dev, s));
    return 0;
}

// Test hook (blt_debug_set_finish): 0 disables the finish kernels (the chain's ordinary passes only).
std::atomic<int> g_finish{1};

// A device error flagged during a general map's chain: the sticky message, with the control
// block's flags and first-error record when they survive.  The u16 scan passes keep them (their
// chunk-map kernel resets only the ticket); a generic u16 pass (merge_tokens_kernel, chunks under
// kTokRange tokens) zeroes the whole control block before its launch, so an error flagged earlier in
// the chain is reported by the sticky message alone.
int chain_sticky(const blt_bpe* h, uint8_t* ws, const WsLayout& L, uint64_t passes) {
    if (!sticky_check(h)) return 0;
    const std::string sticky_msg = t_err;
    uint32_t ctl[16] = {0};
    if (hipMemcpy(ctl, ws + L.ctl, sizeof ctl, hipMemcpyDeviceToHost) == hipSuccess && ctl_error(ctl))
        return fail(BLT_E_IO, "%s; u16 passes 1..%llu: %s", sticky_msg.c_str(), (unsigned long long)passes, t_err.c_str());
    return fail(BLT_E_IO, "%s", sticky_msg.c_str());
}

// Sparse passes of a cyclic map (blt::launch_sparse_*; bpe_kernels.hip explains why they are the
// greedy passes), tried once per encode: enqueued right behind the byte pass (no fused kernel) for
// maps whose byte pass cannot end the chain, else at the first read of the pass counts whose last
// pass merged under 1/16 of its tokens.
// On selfval (256 MiB): 0.85 ms against 1.01 behind the fused passes 1 + 2 and 1.34 with full
// passes only: the byte pass and one more sparse pass (u16 pass 1's ~60 K merges) cost less than
// the fused kernel.  Test hook blt_debug_set_sparse(0) turns them off (full passes only, the fused
// kernel where it applies).
std::atomic<int> g_sparse{1};
// Test hook: sparse passes the calling thread's last general-map encode ran (blt_debug_last_sparse):
// passes | 1 << 16 when they reached the fixpoint, | 1 << 17 when a list overflowed.
thread_local uint32_t t_last_sparse = 0;
// Test hook (blt_debug_set_sparse_cap): the lists' capacity clamped (0: the workspace's), to take the
// not-taken path.
std::atomic<uint32_t> g_sparse_cap{0};

struct SparseRun {
    bool gated = false;      // the chain had ended (or the fused kernel must fall back): nothing ran
    bool taken = false;      // detect found few enough seeds: the passes ran
    bool complete = false;   // ... to the fixpoint (else the full passes go on from the compaction)
    uint32_t passes = 0;     // passes enqueued: the compaction wrote the total as pass k + passes - 1's
    uint32_t applied = 0;    // passes that did work: up to the last with seeds, before any overflow
    uint64_t rec[4] = {0, 0, 0, 0};   // the chain block's totals, done and fallback words, as read last
    bool rec_final = false;  // ... read after the compaction
};

// Host words of the sparse passes' reads (pinned: the reads sit between the device's launches),
// from the handle's free list (blt_bpe::sp_free); a failed allocation leaves the sparse passes out
// of that encode (the full passes give the same tokens).
struct SparseHost {
    uint32_t ctr[kSparseCtrWords];
    uint64_t rec[4];
};
struct SparseHostLease {
    const blt_bpe* h;
    SparseHost* p = nullptr;
    explicit SparseHostLease(const blt_bpe* hh) : h(hh) {
        {
            std::lock_guard<std::mutex> lk(h->sp_mu);
            if (!h->sp_free.empty()) {
                p = static_cast<SparseHost*>(h->sp_free.back());
                h->sp_free.pop_back();
            }
        }
        if (!p && hipHostMalloc(reinterpret_cast<void**>(&p), sizeof(SparseHost), hipHostMallocDefault) != hipSuccess)
            p = nullptr;
    }
    ~SparseHostLease() {
        if (!p) return;
        std::lock_guard<std::mutex> lk(h->sp_mu);
        h->sp_free.push_back(p);
    }
};

// After u16 pass k - 1 (its token count at n_dev on the device, at most n_max, in place in d_out;
// chunk starts off_in): sparse passes k, k + 1, ... in the hole layout, then the compaction into
// d_out, off_out and tot[(k + passes - 1) & 1], as the full passes would leave them.  Enqueued
// without reading anything first: the detect kernel, four passes and the compaction (which runs only
// when the four passes reached the fixpoint and detect's seeds fit the lists), then one read of the
// counters and the chain block.  Passes went on past four: more batches, one read each, then the
// compaction (the caller reads the totals).  Nothing changes when the gate word (done and fallback
// words) is set or detect's seeds overflow the lists (not taken).
// Concurrent runs (threads sharing a handle, several handles, several processes on one device)
// need no coordination: the two kernels whose workgroups wait for other workgroups
// (sparse_list_kernel, sparse_move_kernel) take their work from tickets, so a workgroup only waits
// for lower tickets, held by workgroups that have started (round 5 serialised the batches per
// device with a lock and an event, because those kernels relied on blockIdx dispatch order).
int run_sparse(const blt_bpe* h, const DevTables* t, int dev, hipStream_t s, uint8_t* ws, const WsLayout& L,
               uint8_t* d_out, const uint64_t* n_dev, uint64_t n_max, const uint64_t* gate, uint64_t k,
               const uint64_t* off_in, uint64_t* off_out, uint64_t* tot, SparseRun* r) {
    *r = SparseRun{};
    SparseHostLease lease(h);
    SparseHost* hb = lease.p;
    if (!L.sp_cap || !hb || n_max == 0 || n_max >= (1ull << 32)) return 0;
    if (dev < 0 || dev >= kMaxDevices) return fail(BLT_E_NODEV, "device index %d out of range", dev);
    uint32_t* ctr = reinterpret_cast<uint32_t*>(ws + L.sp_ctr);
    blt::SparseParams q{};
    q.tok = reinterpret_cast<uint16_t*>(d_out);
    q.n = n_max;
    q.n_dev = n_dev;
    q.gate = gate;
    q.holes = reinterpret_cast<uint32_t*>(ws + L.sp_holes);
    q.flags = ctr;
    q.merges = reinterpret_cast<uint32_t*>(ws + L.sp_merges);
    const uint32_t cap_over = g_sparse_cap.load(std::memory_order_relaxed);
    q.cap = cap_over ? std::min(cap_over, L.sp_cap) : L.sp_cap;
    q.hbuckets = t->hbuckets;
    q.hmul1 = h->hmul1;
    q.hmul2 = h->hmul2;
    q.hshift = h->hshift;
    q.hbytes = (uint32_t)(h->hwords.size() * sizeof(uint32_t));
    q.hone = h->hone ? 1u : 0u;
    q.coff_in = off_in;
    q.coff_out = off_out;
    q.nchunks = L.nchunks;
    q.tile_cnt = reinterpret_cast<uint32_t*>(ws + L.sp_tileo);   // (8 B per tile: the counts padded to 16, the total)
    q.super_cnt = q.tile_cnt + ((L.sp_ntiles + 15) & ~15ull);
    q.status = reinterpret_cast<uint64_t*>(ws + L.sp_status);
    // counters, tile counts and status words: zeroed by the first sparse kernel (a memset is one
    // more launch, ~5 us; two when its size is not whole 16-byte units)
    q.zero = reinterpret_cast<uint4*>(ws + L.sp_tileo);
    q.zero16 = (uint32_t)(((L.sp_ctr - L.sp_tileo) + up16(4ull * kSparseCtrWords)) / 16);
    q.sample = reinterpret_cast<uint32_t*>(ws + L.sp_ctr + up16(4ull * kSparseCtrWords));
    q.ctl = reinterpret_cast<uint32_t*>(ws + L.ctl);
    q.sticky = h->sticky.load(std::memory_order_acquire);
    q.inject = g_inject.load(std::memory_order_relaxed);
    uint32_t* seeds[2] = {reinterpret_cast<uint32_t*>(ws + L.sp_seeds0), reinterpret_cast<uint32_t*>(ws + L.sp_seeds1)};
    uint32_t* bits0 = reinterpret_cast<uint32_t*>(ws + L.sp_bits0);
    uint32_t* bits[2] = {reinterpret_cast<uint32_t*>(ws + L.sp_bits1), reinterpret_cast<uint32_t*>(ws + L.sp_bits2)};
    // pass p reads list p & 1 (pass 0's from sparse_list_kernel); its seed bitmap is detect's bits0
    // for pass 0, then bits[(p - 1) & 1], which pass p - 1 wrote (and pass p's apply kernel clears)
    // list slices: one per wave of the region kernel, at least 256 entries each (small inputs run
    // fewer waves)
    {
        uint32_t nsl = std::min<uint32_t>(blt::kSparseSlices, (q.cap / 256u) & ~3u);
        if (nsl < 4) nsl = 4;
        q.nslices = nsl;
        q.slice = q.cap / nsl;
    }
    uint32_t* cnts = reinterpret_cast<uint32_t*>(ws + L.sp_slices);
    q.cnt_merges = cnts + 2 * blt::kSparseSlices;
    auto at_pass = [&](uint32_t pp) {   // pass pp's lists and counters
        q.cnt_in = pp ? cnts + ((pp - 1) & 1) * blt::kSparseSlices : nullptr;
        q.cnt_seeds = cnts + (pp & 1) * blt::kSparseSlices;
        q.seeds_in = seeds[pp & 1];
        q.bits_in = pp ? bits[(pp - 1) & 1] : bits0;
        q.nseeds_in = ctr + 2 + pp;
        q.seeds_out = seeds[(pp + 1) & 1];
        q.bits_out = bits[pp & 1];
        q.bits_alt = bits[1];
        q.nseeds_out = ctr + 2 + pp + 1;
        q.nmerges = ctr + 2 + (kSparseMaxPasses + 1) + pp;
        q.first_pass = pp == 0 ? 1u : 0u;
    };
    const uint32_t* nseeds0 = ctr + 2;
    at_pass(0);
    HIP_TRY(blt::launch_sparse_detect(q, s));
    {   // pass 0's list: bits0 into list 0, counter ctr[2]
        blt::SparseParams ql = q;
        ql.seeds_out = seeds[0];
        ql.nseeds_out = ctr + 2;
        HIP_TRY(blt::launch_sparse_list(ql, s));
    }
    constexpr uint32_t kFirst = 4;
    uint32_t pp = 0;
    for (; pp < kFirst; ++pp) {
        at_pass(pp);
        HIP_TRY(blt::launch_sparse_pass(q, s));
    }
    q.cond = ctr + 2 + kFirst;   // pass kFirst's seeds: none = the fixpoint
    q.total = tot + ((k + kFirst - 1) & 1);
    HIP_TRY(blt::launch_sparse_compact(q, nseeds0, s));
    uint32_t* c = hb->ctr;
    // passes that did work, of the pp enqueued: those before the first that overflowed a list (its
    // merges were dropped and every later region kernel returned at once), and of those the ones up
    // to the last that had seeds (a pass without seeds merges nothing)
    auto applied = [&](uint32_t npass) {
        uint32_t a = 0;
        for (uint32_t p = 0; p < npass; ++p) {
            if (c[2 + (kSparseMaxPasses + 1) + p] > q.cap || c[2 + p + 1] > q.cap) break;
            if (c[2 + p] == 0) break;
            a = p + 1;
        }
        return a;
    };
    HIP_TRY(hipMemcpyAsync(c, ctr, sizeof hb->ctr, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(hb->rec, tot, 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::copy(hb->rec, hb->rec + 4, r->rec);
    if (r->rec[2]) {   // (the gate: done or fallback words)
        r->gated = true;
        return 0;
    }
    if (c[0] & 2u) return 0;   // not taken: the first pass overflowed the lists, nothing was applied
    r->taken = true;
    bool overflow = c[0] != 0;
    if (c[2 + kFirst] == 0) {   // the compaction ran
        r->rec_final = true;
        r->passes = kFirst;
        r->applied = applied(kFirst);
        r->complete = !overflow;
        t_last_sparse = kFirst | (r->complete ? 1u << 16 : 0u) | (overflow ? 1u << 17 : 0u);
        return 0;
    }
    while (!overflow && c[2 + pp] != 0 && pp < kSparseMaxPasses) {   // (the seeds of pass pp, the next to run)
        const uint32_t e = std::min<uint32_t>(pp + 8, kSparseMaxPasses);
        for (; pp < e; ++pp) {
            at_pass(pp);
            HIP_TRY(blt::launch_sparse_pass(q, s));
        }
        HIP_TRY(hipMemcpyAsync(c, ctr, sizeof hb->ctr, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        overflow = c[0] != 0;
    }
    r->passes = pp;
    r->applied = applied(pp);
    r->complete = !overflow && c[2 + pp] == 0;
    q.cond = nullptr;
    q.total = tot + ((k + pp - 1) & 1);
    HIP_TRY(blt::launch_sparse_compact(q, nseeds0, s));
    t_last_sparse = pp | (r->complete ? 1u << 16 : 0u) | (overflow ? 1u << 17 : 0u);
    return 0;
}

int encode_device(const blt_bpe* h, const uint8_t* d_in, uint64_t n, uint64_t cs, uint8_t* d_out,
                  uint64_t* d_chunk_off, void* d_ws, size_t ws_bytes, hipStream_t s, uint64_t* out_tokens,
                  uint32_t flags = 0) {
    if (!h || (!d_in && n) || (!d_out && n)) return fail(BLT_E_INVALID_INPUT, "null argument");
    if (cs == 0) return fail(BLT_E_INVALID_INPUT, "chunk_size must be > 0");
    if (((uintptr_t)d_in | (uintptr_t)d_out | (uintptr_t)d_ws) & 15)
        return fail(BLT_E_INVALID_INPUT, "device buffers must be 16-byte aligned");
    if (n == 0) {
        if (out_tokens) *out_tokens = 0;
        if (d_chunk_off) HIP_TRY(hipMemsetAsync(d_chunk_off, 0, sizeof(uint64_t), s));
        return 0;
    }
    const WsLayout L = ws_layout(h, n, cs);
    if (ws_bytes < L.bytes) return fail(BLT_E_INVALID_INPUT, "workspace too small (%zu < %llu)", ws_bytes, (unsigned long long)L.bytes);
    int dev;
    if (int rc = current_device(&dev)) return rc;
    if (!sticky_word(h)) return fail(BLT_E_NOMEM, "cannot allocate the pinned error word");
    if (int rc = sticky_check(h)) return rc;
    DevTables* t;
    if (int rc = device_tables(h, dev, &t)) return rc;
    uint8_t* ws = static_cast<uint8_t*>(d_ws);

    if (h->single_pass) {
        if (int rc = run_pass(h, t, dev, s, ws, L, d_in, false, n, cs, nullptr, d_out, true, 2 * n, d_chunk_off,
                              (flags & BLT_ENCODE_WORKSPACE_ZEROED) != 0))
            return rc;
        if (out_tokens) {
            if (int rc = read_u64(ws + L.total, out_tokens, s)) return rc;
            return check_ctl(ws, s);
        }
        return 0;
    }

    // General map: pass 1 on bytes into d_out, then passes on big-endian u16 tokens, in place in
    // d_out, until one merges nothing (tokenizer.rs:63-86; a pass that merges nothing leaves the
    // tokens, so running it for every chunk once the slowest chunk is done changes nothing).  The
    // chunk offsets alternate between two arrays.  The host enqueues a batch of passes at a time and
    // reads the pass totals and the done flag once per batch (passes after the done one return at
    // once).  u16 pass k runs on the scan kernel while every chunk holds >= kTokRange tokens
    // (a pass at most halves a chunk: chunk_size >> k), else on the generic kernel.  The scan
    // kernel also ends the chain after a pass none of whose merges made a key component, so
    // most maps finish after one u16 pass: the first batch is 1 pass, later ones 4.  The done
    // word holds the pass k after which nothing merges; its totals and chunk offsets are [k & 1].
    if (L.nchunks >= (1ull << 32)) return fail(BLT_E_INVALID_INPUT, "too many chunks");
    uint64_t* off[2] = {d_chunk_off ? d_chunk_off : reinterpret_cast<uint64_t*>(ws + L.off_a),
                        reinterpret_cast<uint64_t*>(ws + L.off_b)};
    uint64_t* tot = reinterpret_cast<uint64_t*>(ws + L.total);
    uint32_t* done = reinterpret_cast<uint32_t*>(ws + L.total + 16);
    // pass 1's control block and status words and the chain's totals are contiguous: one memset
    // (BLT_ENCODE_WORKSPACE_ZEROED is ignored here, as the header says)
    HIP_TRY(hipMemsetAsync(ws, 0, L.zero_bytes + kChainBlock, s));
    t_last_scan_passes = 0;
    const bool bounded = chain_bounded(h);
    // Passes 1 and 2 in one kernel (run_fused) when the bucket table fits in LDS, chunks hold whole
    // wave ranges, and the first pass need not end the chain itself (maps with byte-pair keys only
    // keep the byte pass, which can); its halo fallback is read where the host reads the chain's
    // totals anyway, so an async bounded chain keeps the two-kernel path.
    // (a cyclic map whose byte pass cannot end the chain takes the sparse passes right behind the
    // byte pass instead: see g_sparse)
    const bool sp_on = L.sp_cap && g_sparse.load(std::memory_order_relaxed) != 0;
    const bool fused = !(flags & kEncodeNoFused) && g_fused.load(std::memory_order_relaxed) && !h->live_first &&
                       !sp_on && !h->byte_self_pair &&
                       h->hwords.size() * sizeof(uint32_t) <= blt::kHashLdsMax && cs >= blt::kMinChunkBytes &&
                       (!bounded || out_tokens != nullptr);
    uint32_t* fused_fail = reinterpret_cast<uint32_t*>(ws + L.total + 20);   // beside the done word
    int cur = 0;
    uint64_t k = 1;   // u16 passes enqueued
    if (fused) {
        if (int rc = run_fused(h, t, dev, s, ws, L, d_in, n, cs, d_out, off[1], tot + 1, done, fused_fail)) return rc;
        cur = 1;
        k = 2;
        if (g_fused_only.load(std::memory_order_relaxed) && out_tokens) {   // (test hook)
            uint32_t ff = 0;
            HIP_TRY(hipMemcpyAsync(&ff, fused_fail, sizeof ff, hipMemcpyDeviceToHost, s));
            if (int rc = read_u64(tot + 1, out_tokens, s)) return rc;
            t_last_fused = ff ? 2 : 1;   // 2: a halo without a restart, the output is not defined
            return 0;
        }
        if (bounded && h->chain_depth > 2) {
            // more passes to enqueue: see first whether the fused kernel resolved every range (a
            // failed one leaves them no-ops, but each costs its launch)
            uint32_t ff = 0;
            HIP_TRY(hipMemcpyAsync(&ff, fused_fail, sizeof ff, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (int rc = chain_sticky(h, ws, L, 1)) return rc;
            if (ff) {
                const int rc = encode_device(h, d_in, n, cs, d_out, d_chunk_off, d_ws, ws_bytes, s, out_tokens,
                                             flags | kEncodeNoFused);
                t_last_fused = 2;
                return rc;
            }
        }
    } else {   // pass 1 (pass id 0): with byte-pair keys it marks itself final when it made no key component
        const Chain c0{nullptr, tot, done, 0};
        if (int rc = run_pass(h, t, dev, s, ws, L, d_in, false, n, cs, nullptr, d_out, true, 2 * n, off[0], true, &c0))
            return rc;
    }
    // a wave range the fused kernel could not resolve: the two-kernel chain from the start
    auto fallback = [&]() {
        const int rc = encode_device(h, d_in, n, cs, d_out, d_chunk_off, d_ws, ws_bytes, s, out_tokens, flags | kEncodeNoFused);
        t_last_fused = 2;
        return rc;
    };
    t_last_fused = fused ? 1 : 0;
    uint64_t rec[4] = {0, 0, 0, 0};
    // what the previous launch left for the next u16 pass (run_pass)
    U16Run u16run;
    // the finish kernels, once per encode: at the first u16 pass whose input chunks may fit in LDS
    bool fin_tried = !g_finish.load(std::memory_order_relaxed);
    auto finish_now = [&](uint64_t kk) {
        if (fin_tried || kk >= 64 || (cs >> kk) > blt::kFinCapTokens) return false;
        fin_tried = true;
        return true;
    };
    if (bounded) {
        // a bounded chain (no value can be made from itself): u16 passes 1 .. depth - 1 are all a
        // pass can need, enqueued without reading the device's pass count; passes after the one
        // that marks the fixpoint return at once, and a last kernel picks the final pass's total
        // and chunk offsets.  Only a caller asking for the token count waits (once).
        const uint32_t k_last = h->chain_depth - 1;
        for (; k <= k_last; ++k) {
            const Chain c{tot + ((k - 1) & 1), tot + (k & 1), done, (uint32_t)k,
                          k + 1 <= k_last && k + 1 < 64 && (cs >> (k + 1)) >= blt::kTokRange};
            if (finish_now(k)) {
                if (int rc = run_finish(h, t, dev, s, ws, L, d_out, (uint32_t)k, off[cur], off[cur ^ 1], tot + (k & 1), done))
                    return rc;
                u16run.reset();
                if (out_tokens) {
                    // a caller that waits anyway: see whether the finish ran (its gate word, the longest
                    // chunk, fit in LDS) before enqueueing the passes it turned into no-ops
                    uint32_t lmax = 0;
                    HIP_TRY(hipMemcpyAsync(&lmax, ws + L.total + 32, sizeof lmax, hipMemcpyDeviceToHost, s));
                    HIP_TRY(hipStreamSynchronize(s));
                    if (lmax <= blt::kFinCapTokens) break;
                }
            }
            const bool scan = k < 64 && (cs >> k) >= blt::kTokRange;
            if (int rc = run_pass(h, t, dev, s, ws, L, d_out, true, n, 0, off[cur], d_out, true, 2 * n, off[cur ^ 1],
                                  false, &c, scan, &u16run))
                return rc;
            cur ^= 1;
        }
        uint64_t* tot_final = tot + 3;   // the chain block's last word
        HIP_TRY(blt::launch_chain_final(tot, done, off[1], d_chunk_off, L.nchunks, k_last, tot_final, s));
        if (!out_tokens) return 0;
        HIP_TRY(hipMemcpyAsync(rec, tot, 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (int rc = chain_sticky(h, ws, L, k_last)) return rc;
        if (fused && (rec[2] >> 32)) return fallback();
        const uint32_t kd = (uint32_t)rec[2];
        t_last_u16_passes = kd ? (kd & ~blt::kDoneBytePass) : k_last;
        *out_tokens = rec[3];
        return 0;
    }
    // sparse passes: tried once, right behind the byte pass or at a read of the pass counts; once
    // more at a read of the pass counts when the try behind the byte pass found its lists too small
    // (cyclic_dense: every word start a seed at first, a few long words at the end)
    bool sp_tried = !sp_on, sp_retry = false;
    t_last_sparse = 0;
    // Before pass k the chain's arrays follow k: its input total is tot[(k - 1) & 1] and it writes
    // tot[k & 1].  The chunk offsets follow cur, which a sparse run flips once whatever number of
    // passes it ran: pass k reads off[cur] = off[((k - 1) & 1) ^ off_shift] and writes the other.
    uint32_t off_shift = 0;
    // passes enqueued that did nothing (a sparse run's passes after its fixpoint or its overflow):
    // k counts them (the compaction wrote its total as the last enqueued pass's), the pass counts
    // reported and checked do not
    uint64_t k_idle = 0;
    // a sparse run that was taken: the passes it ran, then the compaction's results, or the end
    auto sparse_taken = [&](const SparseRun& r, bool* finished) -> int {
        *finished = false;
        cur ^= 1;
        k += r.passes;
        k_idle += r.passes - r.applied;
        off_shift = (uint32_t)cur ^ (uint32_t)((k - 1) & 1);
        if (!r.rec_final) {   // (the totals to read)
            HIP_TRY(hipMemcpyAsync(rec, tot, 32, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
        } else {
            std::copy(r.rec, r.rec + 4, rec);
        }
        if (int rc = chain_sticky(h, ws, L, k - 1 - k_idle)) return rc;
        if (!r.complete) return 0;
        *finished = true;
        t_last_u16_passes = (uint32_t)(k - 1 - k_idle);
        if (d_chunk_off && off[cur] != d_chunk_off)
            HIP_TRY(hipMemcpyAsync(d_chunk_off, off[cur], 8 * (L.nchunks + 1), hipMemcpyDeviceToDevice, s));
        if (out_tokens) *out_tokens = rec[(k - 1) & 1];
        return 0;
    };
    if (sp_on && !bounded && !h->live_first) {   // (no fused kernel: see fused above)
        sp_tried = true;
        SparseRun r;
        const uint64_t* gate = reinterpret_cast<const uint64_t*>(done);   // done word | fallback word
        if (int rc = run_sparse(h, t, dev, s, ws, L, d_out, tot + ((k - 1) & 1), n, gate, k, off[cur], off[cur ^ 1],
                                tot, &r))
            return rc;
        u16run.reset();
        if (r.taken) {
            bool fin = false;
            if (int rc = sparse_taken(r, &fin)) return rc;
            if (fin) return 0;
        } else if (!r.gated) {
            sp_retry = true;
        }
    }
    // A lower bound of the chunks' token counts (the last chunk's aside) beyond cs >> k: min_in for
    // the input of pass min_k, read from the chunk offsets at a batch end; a pass at most halves a
    // chunk.  It keeps the scan kernel on chunks that stay long (cyclic_dense: one letter per word
    // and pass, 16 MiB chunks of ~9 M tokens) past the pass where cs >> k falls below kTokRange, in
    // place of merge_tokens_kernel at twice the time per pass.  (The scan still checks: two chunk
    // starts or ends in one wave range flag error bit 16.)
    uint64_t min_in = 0, min_k = 0;
    std::vector<uint64_t> hoff;
    const int u16c = g_u16_chain.load(std::memory_order_relaxed);
    auto scan_ok = [&](uint64_t kk) {
        if (kk >= 64) return false;
        if ((cs >> kk) >= blt::kTokRange) return true;
        if (!(u16c & 2)) return false;
        return min_in && kk >= min_k && kk - min_k < 64 && (min_in >> (kk - min_k)) >= blt::kTokRange;
    };
    for (int batch = 1;; batch = 4) {
        for (int b = 0; b < batch; ++b, ++k) {
            const Chain c{tot + ((k - 1) & 1), tot + (k & 1), done, (uint32_t)k, scan_ok(k + 1)};
            if (finish_now(k)) {
                if (int rc = run_finish(h, t, dev, s, ws, L, d_out, (uint32_t)k, off[cur], off[cur ^ 1], tot + (k & 1), done))
                    return rc;
                u16run.reset();
            }
            const bool scan = scan_ok(k);
            if (int rc = run_pass(h, t, dev, s, ws, L, d_out, true, n, 0, off[cur], d_out, true, 2 * n, off[cur ^ 1],
                                  false, &c, scan, &u16run))
                return rc;
            cur ^= 1;
        }
        HIP_TRY(hipMemcpyAsync(rec, tot, 32, hipMemcpyDeviceToHost, s));
        // the chunk offsets too when the next batch would leave the scan kernel by cs >> k alone
        // (a few chunks: one more small copy in the same wait)
        const bool rd_off = !scan_ok(k + 4) && L.nchunks >= 2 && L.nchunks <= 4096;
        if (rd_off) {
            hoff.resize(L.nchunks + 1);
            HIP_TRY(hipMemcpyAsync(hoff.data(), off[cur], 8 * (L.nchunks + 1), hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(hipStreamSynchronize(s));
        if (int rc = chain_sticky(h, ws, L, k - 1 - k_idle)) return rc;
        if (fused && (rec[2] >> 32)) return fallback();
        if ((uint32_t)rec[2]) break;
        if (rd_off) {   // pass k's input chunks, the last aside
            uint64_t m = ~0ull;
            for (uint64_t c = 0; c + 1 < L.nchunks; ++c) m = std::min(m, hoff[c + 1] >= hoff[c] ? hoff[c + 1] - hoff[c] : 0);
            min_in = m;
            min_k = k;
        }
        if (k - k_idle > n + 8)
            return fail(BLT_E_IO, "general map: no fixpoint after %llu passes", (unsigned long long)(k - k_idle));
        // the last pass k - 1 left N tokens out of Nin (Nin unknown after the fused passes): the sparse
        // passes are tried once that pass merged under 1/16 of its tokens.  (Under half of what the
        // lists hold, a batch earlier on cyclic_dense, measured slower: 2.35 -> 3.50-3.57 ms.)
        const uint64_t N = rec[(k - 1) & 1], Nin = (k >= 3 || !fused) ? rec[k & 1] : 0;
        if ((!sp_tried || sp_retry) && Nin >= N && (Nin - N) * 16 < N) {
            sp_tried = true;
            sp_retry = false;
            SparseRun r;
            if (int rc = run_sparse(h, t, dev, s, ws, L, d_out, tot + ((k - 1) & 1), N, nullptr, k, off[cur],
                                    off[cur ^ 1], tot, &r))
                return rc;
            u16run.reset();
            if (r.taken) {
                bool fin = false;
                if (int rc = sparse_taken(r, &fin)) return rc;
                if (fin) return 0;
            }
        }
    }
    const uint32_t kdone = (uint32_t)rec[2] & ~blt::kDoneBytePass;   // 0: pass 1 was final
    t_last_u16_passes = (uint32_t)(kdone ? kdone - k_idle : 0);
    const uint32_t last = kdone & 1u;              // the total the final pass wrote
    const uint32_t olast = last ^ off_shift;       // and its chunk offsets (not off[last]
                                                   // after a sparse run of an even number of passes)
    if (d_chunk_off && off[olast] != d_chunk_off)
        HIP_TRY(hipMemcpyAsync(d_chunk_off, off[olast], 8 * (L.nchunks + 1), hipMemcpyDeviceToDevice, s));
    if (out_tokens) *out_tokens = rec[last];
    return 0;
}

// ---- per-device staging contexts for the host-buffer API ---------------------------------
// One slot of the pipelined host path: device buffers for a window of whole chunks, its own
// stream, a pinned record of the window's token count, control words and chunk offsets.
struct PipeSlot {
    hipStream_t stream = nullptr;
    hipEvent_t counted = nullptr;     // the window's kernel and record copy are done
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* d_ws = nullptr;
    uint64_t* d_off = nullptr;
    uint64_t* h_rec = nullptr;        // pinned: [0] tokens, [1..8] control words, [9..] chunk offsets
    uint8_t* h_in = nullptr;          // pinned staging ring (BLT_PIN_RING): the window's bytes,
    uint8_t* h_out = nullptr;         // and its tokens
    uint64_t win = 0, ws_bytes = 0, nch = 0, pin = 0;
};
#ifndef BLT_PIPE_SLOTS
#define BLT_PIPE_SLOTS 4
#endif
#ifndef BLT_PIPE_WIN_MIB
#define BLT_PIPE_WIN_MIB 32
#endif
constexpr int kPipeSlots = BLT_PIPE_SLOTS;
constexpr uint64_t kPipeWindow = (uint64_t)BLT_PIPE_WIN_MIB << 20;   // bytes per window, whole chunks

struct DevCtx {
    int device = 0;
    PipeSlot pipe[kPipeSlots];
    hipStream_t stream = nullptr;
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* d_out = nullptr;
    size_t out_cap = 0;
    uint8_t* d_ws = nullptr;
    size_t ws_cap = 0;
    uint64_t* d_off = nullptr;
    size_t off_cap = 0;
};

std::mutex g_pool_mu;
std::vector<DevCtx*> g_pool;  // idle contexts; never freed (process lifetime)

DevCtx* ctx_acquire(int dev) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (g_pool[i]->device == dev) {
                DevCtx* c = g_pool[i];
                g_pool.erase(g_pool.begin() + (long)i);
                return c;
            }
    }
    DevCtx* c = new DevCtx();
    c->device = dev;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return nullptr;
    }
    return c;
}

void ctx_release(DevCtx* c) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    g_pool.push_back(c);
}

int grow(uint8_t** p, size_t* cap, size_t need) {
    if (*cap >= need && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t sz = std::max<size_t>(need, 4096);
    HIP_TRY(hipMalloc(p, sz));
    *cap = sz;
    return 0;
}

struct CtxGuard {
    DevCtx* c;
    ~CtxGuard() { if (c) ctx_release(c); }
};

// Encodes host bytes [in, in + n) (chunk size cs) on device dev into host out in one staging
// round trip; returns tokens and optional per-chunk token offsets (nchunks + 1).
int encode_host_on(const blt_bpe* h, int dev, const uint8_t* in, uint64_t n, uint64_t cs, uint8_t* out,
                   uint64_t* tokens, std::vector<uint64_t>* chunk_off) {
    HIP_TRY(hipSetDevice(dev));
    DevCtx* c = ctx_acquire(dev);
    if (!c) return fail(BLT_E_IO, "cannot create a HIP stream on device %d", dev);
    CtxGuard guard{c};
    const WsLayout L = ws_layout(h, n, cs);
    if (int rc = grow(&c->d_in, &c->in_cap, up16(n))) return rc;
    if (int rc = grow(&c->d_out, &c->out_cap, up16(2 * n))) return rc;
    if (int rc = grow(&c->d_ws, &c->ws_cap, L.bytes)) return rc;
    uint8_t* offp = reinterpret_cast<uint8_t*>(c->d_off);
    if (int rc = grow(&offp, &c->off_cap, 8 * (L.nchunks + 1))) return rc;
    c->d_off = reinterpret_cast<uint64_t*>(offp);
    HIP_TRY(hipMemcpyAsync(c->d_in, in, n, hipMemcpyHostToDevice, c->stream));
    uint64_t ntok = 0;
    if (int rc = encode_device(h, c->d_in, n, cs, c->d_out, c->d_off, c->d_ws, c->ws_cap, c->stream, &ntok)) return rc;
    HIP_TRY(hipMemcpyAsync(out, c->d_out, 2 * ntok, hipMemcpyDeviceToHost, c->stream));
    if (chunk_off) {
        chunk_off->resize(L.nchunks + 1);
        HIP_TRY(hipMemcpyAsync(chunk_off->data(), c->d_off, 8 * (L.nchunks + 1), hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    *tokens = ntok;
    return 0;
}

// Pinned staging ring of the windowed host path, opt-in: BLT_PIN_RING=1 (or
// blt_debug_set_pin_ring).  Each slot holds a pinned copy of its window's bytes and tokens; the
// producer copies the caller's bytes in with kPinCopyThreads threads and the DMA reads pinned memory,
// the drain copies the tokens out the same way after the device-to-host DMA into pinned memory.  Off
// by default: the runtime's own path from pageable memory is no slower.
std::atomic<int> g_pin_ring{-1};   // -1: from the environment at first use
bool pin_ring_on() {
    int v = g_pin_ring.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("BLT_PIN_RING");
        v = (e && *e && strcmp(e, "0") != 0) ? 1 : 0;
        g_pin_ring.store(v, std::memory_order_relaxed);
    }
    return v != 0;
}
#ifndef BLT_PIN_COPY_THREADS
#define BLT_PIN_COPY_THREADS 4
#endif
constexpr int kPinCopyThreads = BLT_PIN_COPY_THREADS;
// memcpy of n bytes on up to kPinCopyThreads threads (pieces of whole 64 KiB, the caller's thread
// takes the first)
void par_memcpy(uint8_t* dst, const uint8_t* src, uint64_t n) {
    constexpr uint64_t kMin = 4ull << 20, kAlign = 64ull << 10;
    const int nt = n < kMin ? 1 : kPinCopyThreads;
    const uint64_t per = ((n + nt - 1) / nt + kAlign - 1) & ~(kAlign - 1);
    std::thread th[kPinCopyThreads];
    for (int t = 1; t < nt; ++t) {
        const uint64_t a = per * t;
        if (a >= n) break;
        th[t] = std::thread([=] { memcpy(dst + a, src + a, std::min(per, n - a)); });
    }
    memcpy(dst, src, std::min(per, n));
    for (int t = 1; t < nt; ++t)
        if (th[t].joinable()) th[t].join();
}

// Grows slot P of c for windows of `win` bytes in chunks of cs (device buffers, stream, event,
// pinned record; the pinned staging ring when `pin`).  Slots are cached with the context for the
// process lifetime.
int pipe_slot_ready(const blt_bpe* h, PipeSlot& P, uint64_t win, uint64_t cs, bool pin = false) {
    const uint64_t nch = (win + cs - 1) / cs;
    const WsLayout L = ws_layout(h, win, cs);
    if (!P.stream) HIP_TRY(hipStreamCreateWithFlags(&P.stream, hipStreamNonBlocking));
    detail_stamp("slot: stream");
    if (!P.counted) HIP_TRY(hipEventCreateWithFlags(&P.counted, hipEventDisableTiming));
    detail_stamp("slot: event");
    if (P.win < win || P.ws_bytes < L.bytes || P.nch < nch) {
        if (P.d_in) (void)hipFree(P.d_in);   // (one allocation: d_out, d_ws, d_off are carved from it)
        if (P.h_rec) (void)hipHostFree(P.h_rec);
        P.d_in = P.d_out = P.d_ws = nullptr;
        P.d_off = P.h_rec = nullptr;
        P.win = P.ws_bytes = P.nch = 0;
        // one device allocation per slot (four separate hipMallocs cost the CLI's start-up ~30 ms
        // over four slots: profiles/r05_cli_phases.json), 256-byte aligned parts
        auto up256 = [](uint64_t x) { return (x + 255) & ~255ull; };
        const uint64_t o_out = up256(win), o_ws = o_out + up256(2 * win), o_off = o_ws + up256(L.bytes);
        uint8_t* base = nullptr;
        HIP_TRY(hipMalloc(&base, o_off + up256(8 * (nch + 1))));
        detail_stamp("slot: device buffer");
        P.d_in = base;
        P.d_out = base + o_out;
        P.d_ws = base + o_ws;
        P.d_off = reinterpret_cast<uint64_t*>(base + o_off);
        HIP_TRY(hipHostMalloc(&P.h_rec, 8 * (9 + nch + 1), hipHostMallocDefault));
        detail_stamp("slot: pinned record");
        P.win = win;
        P.ws_bytes = L.bytes;
        P.nch = nch;
    }
    if (pin && P.pin < win) {
        if (P.h_in) (void)hipHostFree(P.h_in);
        if (P.h_out) (void)hipHostFree(P.h_out);
        P.h_in = P.h_out = nullptr;
        P.pin = 0;
        HIP_TRY(hipHostMalloc(&P.h_in, up16(win), hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&P.h_out, up16(2 * win), hipHostMallocDefault));
        P.pin = win;
    }
    return 0;
}

// The host-buffer path over windows of whole chunks on several device contexts (chunks are
// independent, pipeline.rs:73-81); window w runs on context w % g.  Per context, a producer thread
// copies its windows in and launches their merge scans (up to kPipeSlots in flight), and a drain
// thread copies each window's tokens back to its final place in `out` as soon as every earlier
// window's token count is known: the output is written in chunk order (pipeline.rs:153-192)
// directly, with no gather or pack pass over it afterwards, and the contexts' H2D, kernels and D2H
// overlap.  Single-pass maps run windows of up to kPipeWindow bytes, asynchronously; general maps
// one window per context (their encode waits for its pass count).
struct MultiRun {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> tok;        // per window; kUnset until counted
    std::vector<uint64_t> off;        // token offset of window w, valid for w <= known
    uint64_t known = 0;
    std::vector<uint64_t> launched, drained;   // per context: windows launched / drained
    int rc = 0;
    std::string err;
    static constexpr uint64_t kUnset = ~0ull;
    void fail_once(int code) {   // with t_err set by the caller's thread
        std::lock_guard<std::mutex> lk(mu);
        if (!rc) { rc = code; err = t_err; }
        cv.notify_all();
    }
};

int encode_host_multi(const blt_bpe* h, const std::vector<int>& devs, const uint8_t* in, uint64_t n, uint64_t cs,
                      uint8_t* out, uint64_t* tokens, std::vector<uint64_t>* chunk_off) {
    const uint64_t g = devs.size();
    const uint64_t nchunks = (n + cs - 1) / cs;
    const uint64_t share = (nchunks + g - 1) / g * cs;   // whole chunks per context
    const uint64_t win = h->single_pass ? std::max<uint64_t>(cs, std::min<uint64_t>(kPipeWindow / cs * cs, share)) : share;
    const uint64_t nw = (n + win - 1) / win;
    const uint64_t per_ctx = (nw + g - 1) / g;
    const int slots = (int)std::min<uint64_t>(kPipeSlots, per_ctx);
    const bool pin = pin_ring_on();
    std::vector<DevCtx*> ctx(g, nullptr);
    struct Release {
        std::vector<DevCtx*>& v;
        ~Release() { for (DevCtx* c : v) if (c) ctx_release(c); }
    } release{ctx};
    for (uint64_t d = 0; d < g; ++d) {
        HIP_TRY(hipSetDevice(devs[d]));
        ctx[d] = ctx_acquire(devs[d]);
        if (!ctx[d]) return fail(BLT_E_IO, "cannot create a HIP stream on device %d", devs[d]);
        // the first slot now, the others by the producer just before their first window: a slot's
        // stream costs ~8-10 ms to create (a hardware queue), off the first window's path
        if (int rc = pipe_slot_ready(h, ctx[d]->pipe[0], std::min(win, n), cs, pin)) return rc;
    }
    MultiRun R;
    R.tok.assign(nw, MultiRun::kUnset);
    R.off.assign(nw + 1, 0);
    R.launched.assign(g, 0);
    R.drained.assign(g, 0);
    if (chunk_off) chunk_off->assign(nchunks + 1, 0);

    auto producer = [&](uint64_t d) {
        DevCtx* c = ctx[d];
        if (hipSetDevice(c->device) != hipSuccess) return R.fail_once(fail(BLT_E_IO, "hipSetDevice(%d) failed", c->device));
        for (uint64_t j = 0, w = d; w < nw; ++j, w += g) {
            {
                std::unique_lock<std::mutex> lk(R.mu);
                R.cv.wait(lk, [&] { return R.rc || R.drained[d] + (uint64_t)slots > j; });
                if (R.rc) return;
            }
            PipeSlot& P = c->pipe[j % slots];
            if (j > 0 && j < (uint64_t)slots)
                if (int rc = pipe_slot_ready(h, P, std::min(win, n), cs, pin)) return R.fail_once(rc);
            const uint64_t b0 = w * win, len = std::min(win, n - b0);
            const WsLayout L = ws_layout(h, len, cs);
            int rc = 0;
            const uint8_t* src = in + b0;
            if (pin) {   // (the slot's pinned copy is free: its window was drained)
                par_memcpy(P.h_in, src, len);
                src = P.h_in;
            }
            if (hipMemcpyAsync(P.d_in, src, len, hipMemcpyHostToDevice, P.stream) != hipSuccess) {
                rc = fail(BLT_E_IO, "host-to-device copy failed on device %d", c->device);
            } else if (h->single_pass) {
                rc = encode_device(h, P.d_in, len, cs, P.d_out, P.d_off, P.d_ws, P.ws_bytes, P.stream, nullptr);
                if (!rc && (hipMemcpyAsync(P.h_rec, P.d_ws + L.total, 8, hipMemcpyDeviceToHost, P.stream) != hipSuccess ||
                            hipMemcpyAsync(P.h_rec + 1, P.d_ws + L.ctl, 64, hipMemcpyDeviceToHost, P.stream) != hipSuccess))
                    rc = fail(BLT_E_IO, "record copy failed on device %d", c->device);
            } else {
                // a general map's chain reads its pass count on the host: the count is final here
                uint64_t ntok = 0;
                rc = encode_device(h, P.d_in, len, cs, P.d_out, P.d_off, P.d_ws, P.ws_bytes, P.stream, &ntok);
                if (!rc) {
                    P.h_rec[0] = ntok;
                    memset(P.h_rec + 1, 0, 64);
                }
            }
            if (!rc && (hipMemcpyAsync(P.h_rec + 9, P.d_off, 8 * (L.nchunks + 1), hipMemcpyDeviceToHost, P.stream) != hipSuccess ||
                        hipEventRecord(P.counted, P.stream) != hipSuccess))
                rc = fail(BLT_E_IO, "record copy failed on device %d", c->device);
            if (rc) return R.fail_once(rc);
            std::lock_guard<std::mutex> lk(R.mu);
            ++R.launched[d];
            R.cv.notify_all();
        }
    };
    struct Pending {
        PipeSlot* P = nullptr;
        uint64_t o = 0, tok = 0;
    };
    auto drain = [&](uint64_t d) {
        DevCtx* c = ctx[d];
        if (hipSetDevice(c->device) != hipSuccess) return R.fail_once(fail(BLT_E_IO, "hipSetDevice(%d) failed", c->device));
        Pending pend;
        auto finish = [&](Pending& q) {   // (pinned ring) window q's tokens into the output, slot released
            if (hipStreamSynchronize(q.P->stream) != hipSuccess) {
                R.fail_once(fail(BLT_E_IO, "device-to-host copy failed on device %d", c->device));
                return false;
            }
            par_memcpy(out + 2 * q.o, q.P->h_out, 2 * q.tok);
            q.P = nullptr;
            std::lock_guard<std::mutex> lk(R.mu);
            ++R.drained[d];
            R.cv.notify_all();
            return true;
        };
        for (uint64_t j = 0, w = d; w < nw; ++j, w += g) {
            {
                std::unique_lock<std::mutex> lk(R.mu);
                R.cv.wait(lk, [&] { return R.rc || R.launched[d] > j; });
                if (R.rc) return;
            }
            PipeSlot& P = c->pipe[j % slots];
            if (hipEventSynchronize(P.counted) != hipSuccess)
                return R.fail_once(fail(BLT_E_IO, "merge scan failed on device %d", c->device));
            uint32_t ctl[16];
            memcpy(ctl, P.h_rec + 1, sizeof ctl);
            if (int rc = ctl_error(ctl)) return R.fail_once(rc);
            const uint64_t tok = P.h_rec[0];
            const uint64_t len = std::min(win, n - w * win), nch = (len + cs - 1) / cs, k0 = w * win / cs;
            uint64_t o = 0;
            {
                std::unique_lock<std::mutex> lk(R.mu);
                R.tok[w] = tok;
                while (R.known < nw && R.tok[R.known] != MultiRun::kUnset) {
                    R.off[R.known + 1] = R.off[R.known] + R.tok[R.known];
                    ++R.known;
                }
                R.cv.notify_all();
                R.cv.wait(lk, [&] { return R.rc || R.known >= w; });   // every earlier window counted
                if (R.rc) return;
                o = R.off[w];
            }
            if (chunk_off)
                for (uint64_t k = 1; k <= nch; ++k) (*chunk_off)[k0 + k] = o + P.h_rec[9 + k];
            if (hipMemcpyAsync(pin ? P.h_out : out + 2 * o, P.d_out, 2 * tok, hipMemcpyDeviceToHost, P.stream) != hipSuccess)
                return R.fail_once(fail(BLT_E_IO, "device-to-host copy failed on device %d", c->device));
            if (pin) {
                // the previous window's tokens out of its pinned copy while this one's DMA runs; this
                // slot is released one window later
                if (pend.P && !finish(pend)) return;
                pend = Pending{&P, o, tok};
                continue;
            }
            std::lock_guard<std::mutex> lk(R.mu);
            ++R.drained[d];
            R.cv.notify_all();
        }
        if (pend.P) (void)finish(pend);
    };
    std::vector<std::thread> th;
    th.reserve(2 * g);
    for (uint64_t d = 0; d < g; ++d) {
        th.emplace_back(producer, d);
        th.emplace_back(drain, d);
    }
    for (auto& t : th) t.join();
    int rc = 0;
    for (uint64_t d = 0; d < g; ++d)
        for (int k = 0; k < slots; ++k)
            if (ctx[d]->pipe[k].stream && hipStreamSynchronize(ctx[d]->pipe[k].stream) != hipSuccess && !rc)
                rc = fail(BLT_E_IO, "device-to-host copy failed on device %d", ctx[d]->device);
    if (R.rc) return fail(R.rc, "%s", R.err.c_str());
    if (rc) return rc;
    *tokens = R.off[nw];
    return 0;
}

// How blt_bpe_process_chunks runs n bytes on n_gpus: device contexts, and the single-staging path
// (encode_host_on) or the windowed one (encode_host_multi).
struct HostPlan {
    std::vector<int> devs;
    bool multi = false;
};
int host_plan(const blt_bpe* h, uint64_t n, uint64_t cs, int n_gpus, HostPlan* plan) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1) return fail(BLT_E_NODEV, "no HIP device available");
    const uint64_t nchunks = (n + cs - 1) / cs;
    // n_gpus device contexts; context d runs on device d % (visible devices), so more contexts than
    // devices share devices (each its own threads and streams).  Windows of whole chunks go to the
    // contexts round-robin and land at their final output offsets in chunk order (encode_host_multi).
    uint64_t g = (uint64_t)std::max(1, std::min(n_gpus < 1 ? 1 : n_gpus, kMaxDevices));
    g = std::min<uint64_t>(g, nchunks);
    // Contexts that would share a device add only contention for its DMA engines and PCIe link
    // (measured on one MI355X: 8 contexts 29.8 GB/s against 45 GB/s for one): one context per
    // device unless a test asks for every shard's own context (blt_debug_set_shared_contexts).
    if (!g_shared_contexts.load(std::memory_order_relaxed)) g = std::min<uint64_t>(g, (uint64_t)count);
    plan->devs.assign(g, 0);
    plan->multi = !(g == 1 && !(h->single_pass && n > kPipeWindow && cs <= kPipeWindow / 2));
    if (g == 1) {
        if (int rc = current_device(&plan->devs[0])) return rc;
    } else {
        for (uint64_t r = 0; r < g; ++r) plan->devs[r] = (int)(r % (uint64_t)count);
    }
    return 0;
}

}  // namespace

// ===========================================================================================
// C ABI
// ===========================================================================================
namespace {

// cgroup CPU quota as num_cpus 1.17 reads it (cgroup v2 cpu.max, v1 cfs quota/period): ceil(quota /
// period), 0 when unlimited or unreadable.
uint64_t cgroup_cpus(const char* root, const char* proc_cgroup) {
    auto read_two = [](const std::string& path, std::string& a, std::string& b) {
        FILE* f = fopen(path.c_str(), "r");
        if (!f) return false;
        char x[64] = {0}, y[64] = {0};
        const int k = fscanf(f, "%63s %63s", x, y);
        fclose(f);
        if (k < 1) return false;
        a = x;
        b = k > 1 ? y : "";
        return true;
    };
    auto ceil_div = [](const std::string& q, const std::string& per) -> uint64_t {
        char* e1 = nullptr;
        char* e2 = nullptr;
        const long long qv = strtoll(q.c_str(), &e1, 10), pv = strtoll(per.c_str(), &e2, 10);
        if (*e1 || *e2 || qv <= 0 || pv <= 0) return 0;
        return (uint64_t)((qv + pv - 1) / pv);
    };
    // the process's own cgroup (v2: "0::/path")
    std::string rel;
    if (FILE* f = fopen(proc_cgroup, "r")) {
        char line[512];
        while (fgets(line, sizeof line, f))
            if (strncmp(line, "0::", 3) == 0) {
                rel = line + 3;
                while (!rel.empty() && (rel.back() == '\n' || rel.back() == '\r')) rel.pop_back();
            }
        fclose(f);
    }
    std::string a, b;
    const std::string r(root);
    for (const std::string& base : {r + (rel == "/" ? "" : rel), r})
        if (read_two(base + "/cpu.max", a, b)) return a == "max" ? 0 : ceil_div(a, b);
    std::string q, per, unused;
    if (read_two(r + "/cpu/cpu.cfs_quota_us", q, unused) && read_two(r + "/cpu/cpu.cfs_period_us", per, unused))
        return ceil_div(q, per);
    return 0;
}

// num_cpus 1.17's logical_cpus(): the CPUs this process may run on (sched_getaffinity), else the
// online CPUs.
uint64_t logical_cpus() {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) {
        const int c = CPU_COUNT(&set);
        if (c > 0) return (uint64_t)c;
    }
    const long c = sysconf(_SC_NPROCESSORS_ONLN);
    return c > 0 ? (uint64_t)c : 1;
}

// num_cpus::get() (utils.rs:79-97 uses it): with a cgroup CPU quota, min(quota, logical_cpus())
// (num_cpus 1.17 init_cgroups; crate not vendored in the reference, restated), else logical_cpus().
uint64_t available_cpus(const char* cgroup_root = "/sys/fs/cgroup", const char* proc_cgroup = "/proc/self/cgroup",
                        uint64_t logical = 0) {
    if (!logical) logical = logical_cpus();
    if (const uint64_t q = cgroup_cpus(cgroup_root, proc_cgroup)) return std::min(q, logical);
    return logical;
}

}  // namespace

extern "C" {

const char* blt_version(void) { return "blt-mi355x 0.2.0"; }

const char* blt_last_error(void) { return t_err.c_str(); }

int blt_load_bpe_merges(const char* path, uint16_t* a, uint16_t* b, uint16_t* v, size_t cap, size_t* n_out) {
    GUARDED(
    if (!path || !n_out) return fail(BLT_E_INVALID_INPUT, "null argument");
    *n_out = 0;
    std::vector<int32_t> table;
    if (int rc = load_merges_table(path, table)) return rc;
    size_t n = 0;
    for (int i = 0; i < 65536; ++i) n += table[i] >= 0;
    *n_out = n;
    if (n > cap) return fail(BLT_E_NOSPC, "need room for %zu entries", n);
    if (n && (!a || !b || !v)) return fail(BLT_E_INVALID_INPUT, "null argument");
    size_t j = 0;
    for (int i = 0; i < 65536; ++i)
        if (table[i] >= 0) {
            a[j] = (uint16_t)(i >> 8);
            b[j] = (uint16_t)(i & 255);
            v[j] = (uint16_t)table[i];
            ++j;
        }
    return 0;
    )
}

int blt_parse_chunk_size(const char* str, uint64_t* out) {
    GUARDED(
    if (!str || !out) return fail(BLT_E_INVALID_INPUT, "null argument");
    // trim (Unicode White_Space, both ends)
    std::string s(str);
    const auto* p = reinterpret_cast<const unsigned char*>(s.data());
    size_t lo = 0, hi = s.size();
    while (lo < hi) {
        uint32_t cp;
        size_t l = utf8_seq(p + lo, hi - lo, &cp);
        if (!l || !is_white_space(cp)) break;
        lo += l;
    }
    while (hi > lo) {
        size_t j = hi - 1;
        while (j > lo && (p[j] & 0xC0) == 0x80) --j;
        uint32_t cp;
        size_t l = utf8_seq(p + j, hi - j, &cp);
        if (!l || l != hi - j || !is_white_space(cp)) break;
        hi = j;
    }
    const std::string t = s.substr(lo, hi - lo);
    if (t.empty()) return fail(BLT_E_INVALID_INPUT, "Input string is empty");
    auto up = [](char c) { return (char)(c >= 'a' && c <= 'z' ? c - 32 : c); };
    const size_t n = t.size();
    const bool unit = n >= 2 && (up(t[n - 2]) == 'K' || up(t[n - 2]) == 'M') && up(t[n - 1]) == 'B';
    const bool digits = std::all_of(t.begin(), t.end(), [](char c) { return c >= '0' && c <= '9'; });
    std::string num;
    uint64_t mult = 1;
    if (unit) {
        num = t.substr(0, n - 2);
        mult = up(t[n - 2]) == 'K' ? 1024ull : 1024ull * 1024ull;
        if (num.empty()) return fail(BLT_E_INVALID_INPUT, "Number part missing for unit '%s'", t.substr(n - 2).c_str());
    } else if (digits) {
        num = t;
    } else {
        return fail(BLT_E_INVALID_INPUT,
                    "Invalid unit or format: '%s'. Number must be followed by KB, MB, or be raw bytes.", t.c_str());
    }
    uint64_t v = 0;
    if (*parse_unsigned(num, UINT64_MAX, &v)) return fail(BLT_E_INVALID_INPUT, "Invalid number: '%s'", num.c_str());
    *out = v * mult;  // release-build wrapping multiply
    return 0;
    )
}

uint64_t blt_effective_chunk_size(int has_cli, uint64_t cli, uint64_t threads, uint32_t memcap) {
    const uint64_t amin = 256ull * 1024, amax = 128ull * 1024 * 1024;
    const uint64_t dmin = 1024ull * 1024, dmax = 16ull * 1024 * 1024;
    if (has_cli) return std::min(std::max(cli, amin), amax);
    const uint64_t usable = (uint64_t)((double)total_ram_bytes() * ((double)memcap / 100.0));
    uint64_t c = usable / std::max<uint64_t>(threads, 1) / 4;
    c = std::min(std::max(c, dmin), dmax);
    return std::min(std::max(c, amin), amax);
}

uint64_t blt_determine_thread_count(int has_cli, uint64_t threads) {
    if (has_cli) return threads == 0 ? 1 : threads;
    return available_cpus();
}

int blt_bpe_create(const uint16_t* a, const uint16_t* b, const uint16_t* v, size_t n, uint32_t flags,
                   blt_bpe** out) {
    GUARDED(
    if (!out || (n && (!a || !b || !v))) return fail(BLT_E_INVALID_INPUT, "null argument");
    if (flags) return fail(BLT_E_INVALID_INPUT, "unknown flags 0x%x", flags);
    std::vector<uint32_t> keys(n);
    std::vector<uint16_t> vals(v, v + n);
    for (size_t i = 0; i < n; ++i) keys[i] = ((uint32_t)a[i] << 16) | b[i];
    return build_handle(keys, vals, out);
    )
}

int blt_bpe_create_from_file(const char* path, blt_bpe** out) {
    GUARDED(
    if (!path || !out) return fail(BLT_E_INVALID_INPUT, "null argument");
    std::vector<int32_t> table;
    if (int rc = load_merges_table(path, table)) {
        // CoreConfig::load_merges_from_file wraps the loader error (lib.rs:194-201)
        const std::string inner = t_err;
        return fail(rc, "Failed to load BPE merges: %s", inner.c_str());
    }
    std::vector<uint32_t> keys;
    std::vector<uint16_t> vals;
    for (uint32_t i = 0; i < 65536; ++i)
        if (table[i] >= 0) { keys.push_back(((i >> 8) << 16) | (i & 255)); vals.push_back((uint16_t)table[i]); }
    return build_handle(keys, vals, out);
    )
}

void blt_bpe_destroy(blt_bpe* h) {
    if (!h) return;
    for (int d = 0; d < kMaxDevices; ++d) {
        if (h->dev[d].dense) (void)hipFree(h->dev[d].dense);   // (the tables' one allocation)
    }
    if (uint32_t* w = h->sticky.load(std::memory_order_acquire)) (void)hipHostFree(w);
    for (void* p : h->sp_free) (void)hipHostFree(p);
    delete h;
}

int blt_bpe_info(const blt_bpe* h, size_t* n_entries, int* single_pass) {
    if (!h) return fail(BLT_E_INVALID_INPUT, "null handle");
    if (n_entries) *n_entries = h->n_entries;
    if (single_pass) *single_pass = h->single_pass ? 1 : 0;
    return 0;
}

int blt_bpe_clear_error(const blt_bpe* h) {
    if (!h) return fail(BLT_E_INVALID_INPUT, "null handle");
    uint32_t* w = h->sticky.load(std::memory_order_acquire);
    if (!w || !__atomic_exchange_n(w, 0u, __ATOMIC_ACQ_REL)) return 0;
    return fail(BLT_E_IO, "a merge scan on this handle had flagged a device error (now cleared)");
}

size_t blt_bpe_workspace_size(const blt_bpe* h, uint64_t n, uint64_t cs) {
    if (!h || cs == 0) return 0;
    return (size_t)ws_layout(h, n, cs).bytes;
}

int blt_bpe_encode_device(const blt_bpe* h, const uint8_t* d_in, uint64_t n, uint64_t cs, uint8_t* d_out,
                          uint64_t* d_chunk_off, void* d_ws, size_t ws_bytes, void* stream, uint64_t* out_tokens) {
    GUARDED(return encode_device(h, d_in, n, cs, d_out, d_chunk_off, d_ws, ws_bytes, (hipStream_t)stream, out_tokens);)
}

int blt_bpe_encode_device_ex(const blt_bpe* h, const uint8_t* d_in, uint64_t n, uint64_t cs, uint8_t* d_out,
                             uint64_t* d_chunk_off, void* d_ws, size_t ws_bytes, void* stream, uint64_t* out_tokens,
                             uint32_t flags) {
    if (flags & ~BLT_ENCODE_WORKSPACE_ZEROED) return fail(BLT_E_INVALID_INPUT, "unknown flags 0x%x", flags);
    GUARDED(
    return encode_device(h, d_in, n, cs, d_out, d_chunk_off, d_ws, ws_bytes, (hipStream_t)stream, out_tokens, flags);
    )
}

int blt_bpe_workspace_reset(const blt_bpe* h, void* d_ws, uint64_t n, uint64_t cs, void* stream) {
    if (!h || !d_ws || cs == 0) return fail(BLT_E_INVALID_INPUT, "bad argument");
    const WsLayout L = ws_layout(h, n, cs);
    HIP_TRY(hipMemsetAsync(d_ws, 0, L.zero_bytes, (hipStream_t)stream));
    // the status words a BLT_ENCODE_WORKSPACE_ZEROED launch may rely on (it refuses beyond them)
    if (L.ntiles <= 0xFFFFFFFFull)
        HIP_TRY(hipMemsetD32Async(static_cast<uint32_t*>(d_ws) + blt::kCtlCover, (int)(uint32_t)L.ntiles, 1,
                                  (hipStream_t)stream));
    return 0;
}

int blt_bpe_check_workspace(void* d_ws, void* stream) {
    if (!d_ws) return fail(BLT_E_INVALID_INPUT, "null workspace");
    hipStream_t s = (hipStream_t)stream;
    if (int rc = check_ctl(static_cast<uint8_t*>(d_ws), s)) {
        const std::string msg = t_err;
        uint32_t z[16] = {0};
        (void)hipMemcpyAsync(d_ws, z, sizeof z, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
        return fail(rc, "%s", msg.c_str());
    }
    return 0;
}

// Not in the public header: the handle's byte-pass choice (tests): byte_mode (-1: the generic byte
// pass) in the low byte, allmerge << 8, live_first << 9.
int blt_debug_byte_mode(const blt_bpe* h) {
    if (!h) return -1;
    return (h->byte_mode & 0xFF) | (h->allmerge ? 0x100 : 0) | (h->live_first ? 0x200 : 0);
}

// Not in the public header (tests): 0 disables the finish kernels of a general map's chain, 1 (the
// default) enables them; returns the previous setting.
int blt_debug_set_finish(int on) { return g_finish.exchange(on ? 1 : 0); }
int blt_debug_set_sparse(int on) { return g_sparse.exchange(on ? 1 : 0); }
uint32_t blt_debug_last_sparse(void) { return t_last_sparse; }
uint32_t blt_debug_set_sparse_cap(uint32_t cap) { return g_sparse_cap.exchange(cap); }

// Not in the public header: a general map's longest merge chain (0: single-pass, or unbounded).
uint32_t blt_debug_chain_depth(const blt_bpe* h) { return h ? h->chain_depth : 0; }

// Not in the public header: a test hook that makes blt_bpe_process_chunks run n_gpus device
// contexts even where several share a device (on a one-GPU box: every context's producer and drain
// threads, sharing the device); 0 restores one context per device.
void blt_debug_set_shared_contexts(int on) { g_shared_contexts.store(on ? 1 : 0, std::memory_order_relaxed); }
// Not in the public header: a test hook for the pinned staging ring of the windowed host path
// (BLT_PIN_RING); returns the previous setting.
int blt_debug_set_pin_ring(int on) { return g_pin_ring.exchange(on ? 1 : 0) > 0 ? 1 : 0; }

// Test hook: 0 runs every general map on the two-kernel chain, 1 (default) lets eligible maps fuse
// passes 1 and 2.
void blt_debug_set_fused(int on) { g_fused.store(on ? 1 : 0, std::memory_order_relaxed); }
int blt_debug_set_u16_chain(int bits) { return g_u16_chain.exchange(bits); }
int blt_debug_set_fused_only(int on) { return g_fused_only.exchange(on ? 1 : 0); }
uint32_t blt_debug_last_fused() { return t_last_fused; }

// Not in the public header: num_cpus::get() over a given cgroup root, /proc/self/cgroup file and
// logical CPU count (tests: fake cgroup trees).
uint64_t blt_debug_available_cpus(const char* cgroup_root, const char* proc_cgroup, uint64_t logical) {
    return available_cpus(cgroup_root, proc_cgroup, logical);
}

// Not in the public header: a test hook that makes every merge pass record, per tile, its
// carry-in/offset/look-back lane and both hypothesis counts into a device buffer.
void blt_debug_set_tile_record(uint64_t* d_buf) { g_debug_tiles = d_buf; }
// Not in the public header: blt::kInject* bits (1 finish kernel, 2 u16 scan, 4 sparse move) the next
// launches break a count with, to check the kernels' invariant checks (returns the old bits).
uint32_t blt_debug_set_inject(uint32_t bits) { return g_inject.exchange(bits); }

// Not in the public header: the number of u16 passes the calling thread's last general-map
// encode ran (the pass after which nothing can merge; later enqueued passes returned at once).
uint32_t blt_debug_last_u16_passes(void) { return t_last_u16_passes; }
// Not in the public header: u16 passes the calling thread's last general-map encode enqueued on the
// scan kernel (done or not).
uint32_t blt_debug_last_scan_passes(void) { return t_last_scan_passes; }

// Not in the public header: a test hook that runs the kernels' device-error path (the one a
// look-back timeout takes) for handle h on the current device and stream, setting error bit 1 in
// d_ws's control block (nullable) and the handle's sticky word.
int blt_debug_inject_device_error(const blt_bpe* h, void* d_ws, void* stream) {
    if (!h) return fail(BLT_E_INVALID_INPUT, "null handle");
    int dev;
    if (int rc = current_device(&dev)) return rc;
    uint32_t* w = sticky_word(h);
    if (!w) return fail(BLT_E_NOMEM, "cannot allocate the pinned error word");
    HIP_TRY(blt::launch_inject_error(static_cast<uint32_t*>(d_ws), w, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}

int blt_basic_encode_device(const uint8_t* d_in, uint64_t n, uint8_t* d_out, void* stream) {
    if ((!d_in || !d_out) && n) return fail(BLT_E_INVALID_INPUT, "null argument");
    if (((uintptr_t)d_in | (uintptr_t)d_out) & 15) return fail(BLT_E_INVALID_INPUT, "device buffers must be 16-byte aligned");
    int dev;
    if (int rc = current_device(&dev)) return rc;
    HIP_TRY(blt::launch_basic_expand(d_in, n, d_out, (hipStream_t)stream));
    return 0;
}

int blt_bpe_process_chunk(const blt_bpe* h, const uint8_t* in, size_t n, uint8_t* out, size_t out_cap,
                          size_t* out_len) {
    GUARDED(
    if (!h || !out_len || (n && (!in || !out))) return fail(BLT_E_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (int rc = sticky_check(h)) return rc;
    if (n == 0) return 0;  // tokenizer.rs:57-59
    if (out_cap < 2 * (uint64_t)n) return fail(BLT_E_NOSPC, "out_cap %zu < 2 * n", out_cap);
    int dev;
    if (int rc = current_device(&dev)) return rc;
    uint64_t ntok = 0;
    if (int rc = encode_host_on(h, dev, in, n, n, out, &ntok, nullptr)) return rc;
    *out_len = 2 * ntok;
    return 0;
    )
}

int blt_basic_process_chunk(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, size_t* out_len) {
    GUARDED(
    if (!out_len || (n && (!in || !out))) return fail(BLT_E_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (n == 0) return 0;  // tokenizer.rs:109-111
    if (out_cap < 2 * (uint64_t)n) return fail(BLT_E_NOSPC, "out_cap %zu < 2 * n", out_cap);
    int dev;
    if (int rc = current_device(&dev)) return rc;
    DevCtx* c = ctx_acquire(dev);
    if (!c) return fail(BLT_E_IO, "cannot create a HIP stream");
    CtxGuard guard{c};
    if (int rc = grow(&c->d_in, &c->in_cap, up16(n))) return rc;
    if (int rc = grow(&c->d_out, &c->out_cap, up16(2 * n))) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_in, in, n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(blt::launch_basic_expand(c->d_in, n, c->d_out, c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->d_out, 2 * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *out_len = 2 * n;
    return 0;
    )
}

}  // extern "C"

// Device setup ahead of a blt_bpe_process_chunks(h, ., n, cs, n_gpus) call (blt_run_tokenizer runs
// it beside the input's mmap): HIP start-up, the handle's device tables and the staging buffers
// that call will use, left in the context pool.  Failures are left for the call itself to report.
void blt_prewarm_chunks(const blt_bpe* h, uint64_t n, uint64_t cs, int n_gpus) try {
    if (!h || !n || !cs) return;
    // BLT_CLI_TIMING: the setup's steps (seconds from this call's start), on stderr
    const bool timing = getenv("BLT_CLI_TIMING") != nullptr;
    timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    auto stamp = [&](const char* what) {
        if (!timing) return;
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        fprintf(stderr, "blt timing: prewarm step: %s +%.4f s\n", what,
                (double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec));
    };
    HostPlan plan;
    if (host_plan(h, n, cs, n_gpus, &plan) != 0) return;
    stamp("device count (runtime up)");
    const uint64_t g = plan.devs.size();
    const uint64_t nchunks = (n + cs - 1) / cs;
    const uint64_t share = (nchunks + g - 1) / g * cs;
    const uint64_t win = h->single_pass ? std::max<uint64_t>(cs, std::min<uint64_t>(kPipeWindow / cs * cs, share)) : share;
    const uint64_t per_ctx = ((n + win - 1) / win + g - 1) / g;
    const int slots = (int)std::min<uint64_t>(kPipeSlots, per_ctx);
    (void)sticky_word(h);
    detail_stamp("sticky word");
    for (uint64_t d = 0; d < g; ++d) {
        const int dev = plan.devs[d];
        if (hipSetDevice(dev) != hipSuccess) return;
        DevCtx* c = ctx_acquire(dev);
        if (!c) return;
        CtxGuard guard{c};
        stamp("context (streams)");
        DevTables* t;
        if (device_tables(h, dev, &t, c->stream) != 0) return;
        stamp("device tables");
        if (plan.multi) {
            // the first slot (blt_bpe_process_chunks readies the others beside its first window)
            if (slots > 0 && pipe_slot_ready(h, c->pipe[0], std::min(win, n), cs) != 0) return;
            stamp("pipeline slots");
            // the code object's load, off the first window's path
            if (blt::launch_noop(c->pipe[0].stream) == hipSuccess) (void)hipStreamSynchronize(c->pipe[0].stream);
            stamp("code object loaded (first launch)");
        } else {
            const WsLayout L = ws_layout(h, n, cs);
            uint8_t* offp = reinterpret_cast<uint8_t*>(c->d_off);
            if (grow(&c->d_in, &c->in_cap, up16(n)) || grow(&c->d_out, &c->out_cap, up16(2 * n)) ||
                grow(&c->d_ws, &c->ws_cap, L.bytes) || grow(&offp, &c->off_cap, 8 * (L.nchunks + 1)))
                return;
            c->d_off = reinterpret_cast<uint64_t*>(offp);
        }
    }
    if (g == 1 && !plan.multi) (void)hipSetDevice(plan.devs[0]);
} catch (...) {
}

extern "C" {

int blt_bpe_process_chunks(const blt_bpe* h, const uint8_t* in, size_t n, size_t cs, int n_gpus, uint8_t* out,
                           size_t out_cap, size_t* out_len, uint64_t* chunk_out_len) {
    GUARDED(
    if (!h || !out_len || (n && (!in || !out))) return fail(BLT_E_INVALID_INPUT, "null argument");
    if (cs == 0) return fail(BLT_E_INVALID_INPUT, "chunk_size must be > 0");
    *out_len = 0;
    if (int rc = sticky_check(h)) return rc;
    if (n == 0) return 0;
    if (out_cap < 2 * (uint64_t)n) return fail(BLT_E_NOSPC, "out_cap %zu < 2 * n", out_cap);
    const uint64_t nchunks = (n + cs - 1) / cs;
    HostPlan plan;
    if (int rc = host_plan(h, n, cs, n_gpus, &plan)) return rc;
    uint64_t total = 0;
    std::vector<uint64_t> offs;
    if (!plan.multi) {
        if (int rc = encode_host_on(h, plan.devs[0], in, n, cs, out, &total, chunk_out_len ? &offs : nullptr)) return rc;
    } else {
        if (int rc = encode_host_multi(h, plan.devs, in, n, cs, out, &total, chunk_out_len ? &offs : nullptr)) return rc;
    }
    if (chunk_out_len)
        for (uint64_t k = 0; k < nchunks; ++k) chunk_out_len[k] = 2 * (offs[k + 1] - offs[k]);
    *out_len = 2 * total;
    return 0;
    )
}

}  // extern "C"
