// run_tokenizer (blt_core/src/lib.rs:246-267) and the chunked pipeline it drives
// (blt_core/src/pipeline.rs:22-433) as one C-ABI entry point, blt_run_tokenizer: the `blt` CLI
// (blt_cli.cpp) and the Python ByteTokenizer.tokenize_file (blt_amd/__init__.py) both call it.
//
// Order of effects as in the reference: the input is opened first (io_handler.rs:55-62: File::open
// + mmap, or stdin), then the output file is created (io_handler.rs:70-78), then the content-type
// token is written (lib.rs:284-293), then the chunks.  Two input paths (pipeline.rs:22-51):
//  * a file is mapped and cut into fixed chunk-size chunks (pipeline.rs:73-81); windows of whole
//    chunks go to blt_bpe_process_chunks / blt_basic_process_chunk (GPU) while the previous window
//    is written, so the output is the chunk outputs concatenated in chunk order (pipeline.rs:153-192);
//  * stdin: one read per chunk (pipeline.rs:303-318).  The reference reads through tokio's stdin,
//    whose blocking adapter (tokio 1.45.1, io/blocking.rs, DEFAULT_MAX_BUF_SIZE) caps one read at
//    2 MiB, so a chunk is one read(2) of at most min(chunk_size, 2 MiB) bytes; a short read makes a
//    short chunk.  Up to `threads` chunks are in flight (pipeline.rs:286) and results are written
//    in chunk order.
// Every error is returned (first one wins), never exit()ed: 0 or a BLT_E_* code with the message in
// blt_last_error().
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <stdarg.h>
#include <strings.h>

#include "../../include/blt_bpe.h"

namespace blt_internal {
int set_error(int code, const char* fmt, ...);
}
using blt_internal::set_error;

// ---- logging (the reference's tracing, src/main.rs:83-85) ----------------------------------
// blt_log_init_from_env sets one level per target this library logs under (blt_core,
// blt_core::pipeline, blt_core::tokenizer) from RUST_LOG (BLT_LOG when unset), the way
// tracing-subscriber 0.3's EnvFilter::from_default_env reads it: a comma list of directives, each
// "level", "target" (every level of it) or "target=level"; a directive applies to a target that
// starts with its own (a bare level to every target), and of those that apply the one with the
// longest target decides (the last such when two are equally long); a target no directive applies
// to logs nothing; a variable that is unset, empty or holds no valid directive means errors only.
// An unknown level after '=' makes that directive invalid (ignored).  Before the call (library users
// other than the CLI, as the Python binding) nothing is logged.  Lines go to stdout with one
// write(2) each (tracing's fmt subscriber writes to stdout; the run's own stdout writes are
// unbuffered too, so the order is the order of the calls).
namespace blt_log {
enum Level { kOff = 0, kError, kWarn, kInfo, kDebug, kTrace };
enum Target { kCore = 0, kPipeline, kTokenizer, kTargets };
const char* const kTargetNames[kTargets] = {"blt_core", "blt_core::pipeline", "blt_core::tokenizer"};
std::atomic<int> g_level[kTargets] = {{-1}, {-1}, {-1}};   // -1: not initialised (nothing is logged)
std::mutex g_mu;

int parse_level(const char* s, size_t n) {
    static const char* names[] = {"off", "error", "warn", "info", "debug", "trace"};
    for (int i = 0; i < 6; ++i)
        if (strlen(names[i]) == n && strncasecmp(s, names[i], n) == 0) return i;
    return -1;
}

// the level of target `t` (kTargetNames) under the directives in v (RUST_LOG's value, nullable)
int level_for(const char* v, int t) {
    const std::string name = kTargetNames[t];
    int valid = 0, level = kOff;
    long spec = -1;   // the deciding directive's target length so far
    for (const char* d = v; d && *d;) {
        const char* e = strchr(d, ',');
        const size_t n = e ? (size_t)(e - d) : strlen(d);
        std::string dir(d, n);
        d = e ? e + 1 : nullptr;
        while (!dir.empty() && dir.back() == ' ') dir.pop_back();
        while (!dir.empty() && dir.front() == ' ') dir.erase(dir.begin());
        if (dir.empty()) continue;
        const size_t eq = dir.find('=');
        std::string target;
        int lv;
        if (eq == std::string::npos) {
            lv = parse_level(dir.data(), dir.size());
            if (lv < 0) {   // a bare target: every level of it
                target = dir;
                lv = kTrace;
            }
        } else {
            target = dir.substr(0, eq);
            lv = parse_level(dir.data() + eq + 1, dir.size() - eq - 1);
            if (lv < 0) continue;   // invalid: ignored
        }
        ++valid;
        if (name.compare(0, target.size(), target) != 0) continue;   // not a prefix of this target
        if ((long)target.size() >= spec) {
            spec = (long)target.size();
            level = lv;
        }
    }
    return valid ? level : (int)kError;
}

int target_of(const char* name) {
    for (int t = 0; t < kTargets; ++t)
        if (strcmp(name, kTargetNames[t]) == 0) return t;
    return kCore;
}
bool on(int lv, int t) { return g_level[t].load(std::memory_order_relaxed) >= lv; }

// "<UTC time>  LEVEL <spans>: <target>: <message>"
void emit(int lv, const char* spans, const char* target, const char* fmt, ...) {
    if (!on(lv, target_of(target))) return;
    static const char* names[] = {"", "ERROR", " WARN", " INFO", "DEBUG", "TRACE"};
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    struct tm tm;
    gmtime_r(&ts.tv_sec, &tm);
    char line[1024];
    int k = snprintf(line, sizeof line, "%04d-%02d-%02dT%02d:%02d:%02d.%06ldZ %s %s%s%s: ", tm.tm_year + 1900,
                     tm.tm_mon + 1, tm.tm_mday, tm.tm_hour, tm.tm_min, tm.tm_sec, ts.tv_nsec / 1000, names[lv],
                     spans ? spans : "", spans && *spans ? ": " : "", target);
    va_list ap;
    va_start(ap, fmt);
    if (k > 0 && (size_t)k < sizeof line) k += vsnprintf(line + k, sizeof line - (size_t)k, fmt, ap);
    va_end(ap);
    if (k < 0) return;
    if ((size_t)k >= sizeof line - 1) k = (int)sizeof line - 2;
    line[k++] = '\n';
    std::lock_guard<std::mutex> g(g_mu);
    for (const char* p = line; k > 0;) {
        const ssize_t w = ::write(1, p, (size_t)k);
        if (w <= 0) {
            if (w < 0 && errno == EINTR) continue;
            return;
        }
        p += w;
        k -= (int)w;
    }
}
}  // namespace blt_log

extern "C" void blt_log_init_from_env(void) {
    const char* v = getenv("RUST_LOG");
    if (!v) v = getenv("BLT_LOG");
    for (int t = 0; t < blt_log::kTargets; ++t) blt_log::g_level[t].store(blt_log::level_for(v, t), std::memory_order_relaxed);
}

namespace {

constexpr size_t kStdinReadCap = size_t(2) << 20;   // tokio io::blocking DEFAULT_MAX_BUF_SIZE

// Debug lines of the chunks [k0, k1) of a file input (pipeline.rs:108 per received result; the
// basic strategy's per-chunk line, tokenizer.rs:113).
void log_chunks(const std::string& span, bool basic, size_t k0, size_t k1, size_t n, size_t cs) {
    if (!blt_log::on(blt_log::kDebug, blt_log::kPipeline) && !(basic && blt_log::on(blt_log::kDebug, blt_log::kTokenizer)))
        return;   // (emit checks each line's own target)
    for (size_t k = k0; k < k1; ++k) {
        if (basic) {
            const std::string sp = span + ":process_mmap_chunk_task{task_id=" + std::to_string(k) +
                                   "}:basic_tokenization_strategy_process";
            blt_log::emit(blt_log::kDebug, sp.c_str(), "blt_core::tokenizer", "Converting %zu bytes to u16 tokens",
                          std::min(cs, n - k * cs));
        }
        blt_log::emit(blt_log::kDebug, span.c_str(), "blt_core::pipeline", "Received result for mmap task task_id=%zu", k);
    }
}

// First error of a run wins; later ones are dropped.
struct RunStatus {
    std::mutex mu;
    int rc = 0;
    std::string msg;
    void set(int code, const std::string& m) {
        std::lock_guard<std::mutex> g(mu);
        if (!rc) { rc = code; msg = m; }
    }
    bool failed() {
        std::lock_guard<std::mutex> g(mu);
        return rc != 0;
    }
};

int os_error(int e) {
    return set_error(e == ENOENT ? BLT_E_NOT_FOUND : BLT_E_IO, "%s (os error %d)", strerror(e), e);
}

std::string last_error() {
    const char* m = blt_last_error();
    return m ? std::string(m) : std::string();
}

// Ordered sink over a file descriptor.  Positioned parallel writes only into an output file this
// run created itself (O_TRUNC, offset 0, nobody else writing it); stdout, whatever it is (pipe,
// terminal, a shared or O_APPEND file), gets plain sequential write()s, so its file offset advances
// exactly as the reference's tokio::io::stdout() writes advance it.
struct Sink {
    int fd = 1;
    bool positioned = false;
    off_t pos = 0;
    static int put(int fd, const uint8_t* p, size_t n, off_t at, bool positioned) {
        while (n) {
            const ssize_t w = positioned ? ::pwrite(fd, p, n, at) : ::write(fd, p, n);
            if (w < 0) {
                if (errno == EINTR) continue;
                return os_error(errno);
            }
            p += w;
            n -= (size_t)w;
            at += w;
        }
        return 0;
    }
    int write_all(const uint8_t* p, size_t n) {
        constexpr size_t kPart = size_t(32) << 20;
        if (!positioned || n < 2 * kPart) {
            const int rc = put(fd, p, n, pos, positioned);
            pos += (off_t)n;
            return rc;
        }
        // page-cache copies of one big write scale with threads
        const size_t parts = std::min<size_t>(8, n / kPart);
        const size_t each = (n / parts + 4095) & ~size_t(4095);
        std::vector<std::thread> th;
        std::vector<int> rcs(parts, 0);
        std::vector<std::string> msgs(parts);
        for (size_t i = 1; i < parts; ++i) {
            const size_t b = i * each;
            if (b >= n) break;
            th.emplace_back([&, i, b] {
                rcs[i] = put(fd, p + b, std::min(each, n - b), pos + (off_t)b, true);
                if (rcs[i]) msgs[i] = last_error();
            });
        }
        int rc = put(fd, p, std::min(each, n), pos, true);
        for (auto& t : th) t.join();
        for (size_t i = 1; i < parts && !rc; ++i)
            if (rcs[i]) rc = set_error(rcs[i], "%s", msgs[i].c_str());
        pos += (off_t)n;
        return rc;
    }
};

// An output buffer that is never zero-filled and keeps its pages between windows.
struct Buf {
    std::unique_ptr<uint8_t[]> p;
    size_t cap = 0, len = 0;
    void reserve(size_t n) {
        if (cap >= n) return;
        p.reset(new uint8_t[n]);
        cap = n;
    }
};

// The per-chunk transform of the selected strategy (lib.rs:271-282, tokenizer.rs:21-31).
struct Strategy {
    enum Kind { kPassthrough, kBpe, kBasic } kind;
    const blt_bpe* h = nullptr;
    int gpus = 1;

    int chunk(const uint8_t* in, size_t n, std::vector<uint8_t>& out) const {
        out.clear();
        if (n == 0) return 0;
        if (kind == kPassthrough) {
            out.assign(in, in + n);
            return 0;
        }
        out.resize(2 * n);
        size_t olen = 0;
        const int rc = kind == kBpe ? blt_bpe_process_chunk(h, in, n, out.data(), out.size(), &olen)
                                    : blt_basic_process_chunk(in, n, out.data(), out.size(), &olen);
        out.resize(rc ? 0 : olen);
        return rc;
    }

    // A window of whole chunks (the last may be short), outputs concatenated in chunk order.
    // Passthrough and basic are position-wise (tokenizer.rs:108-124, :129-137).
    int window(const uint8_t* in, size_t n, size_t cs, Buf& out) const {
        out.len = 0;
        if (n == 0) return 0;
        if (kind == kPassthrough) {
            out.reserve(n);
            memcpy(out.p.get(), in, n);
            out.len = n;
            return 0;
        }
        out.reserve(2 * n);
        size_t olen = 0;
        const int rc = kind == kBpe ? blt_bpe_process_chunks(h, in, n, cs, gpus, out.p.get(), out.cap, &olen, nullptr)
                                    : blt_basic_process_chunk(in, n, out.p.get(), out.cap, &olen);
        out.len = rc ? 0 : olen;
        return rc;
    }
};

// mmap path (pipeline.rs:56-192): windows of whole chunks, window k+1 tokenised while window k is
// written.
int run_mmap(const Strategy& st, const uint8_t* in, size_t n, size_t cs, Sink& sink, const std::string& span) {
    if (n == 0) return 0;
    const size_t per = std::max<size_t>(1, (size_t(256) << 20) / cs);   // ~256 MiB of input per window
    const size_t win = per * cs;
    Buf buf[2];
    std::thread writer;
    int wrc = 0;
    std::string wmsg;
    int rc = 0;
    // BLT_CLI_TIMING: time in the tokenising calls and waiting for the writer, per run
    const bool timing = getenv("BLT_CLI_TIMING") != nullptr;
    double t_tok = 0, t_wait = 0;
    auto now = [] {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
    };
    double t_first = 0;
    for (size_t off = 0, k = 0; off < n && !rc; off += win, ++k) {
        const size_t len = std::min(win, n - off);
        Buf& out = buf[k & 1];
        const double t0 = timing ? now() : 0;
        rc = st.window(in + off, len, cs, out);
        const double t1 = timing ? now() : 0;
        if (writer.joinable()) writer.join();   // window k-1 written: its buffer is free
        if (timing) {
            if (k == 0) t_first = t1 - t0; else t_tok += t1 - t0;
            t_wait += now() - t1;
        }
        if (wrc) break;
        if (rc) break;
        log_chunks(span, st.kind == Strategy::kBasic, off / cs, (off + len + cs - 1) / cs, n, cs);
        writer = std::thread([&sink, &out, &wrc, &wmsg] {
            wrc = sink.write_all(out.p.get(), out.len);
            if (wrc) wmsg = last_error();
        });
    }
    {
        const double t1 = timing ? now() : 0;
        if (writer.joinable()) writer.join();
        if (timing) {
            t_wait += now() - t1;
            fprintf(stderr, "blt timing: %zu window(s) of %zu MiB: first window %.4f s (device setup included), "
                    "tokenise the rest %.4f s, wait for writer %.4f s\n", (n + win - 1) / win, win >> 20, t_first,
                    t_tok, t_wait);
        }
    }
    if (rc) return rc;
    if (wrc) return set_error(wrc, "%s", wmsg.c_str());
    return 0;
}

// Direct path for a regular output file this run created (round 4): the file is sized to the
// output's bound (ftruncate), mapped shared, and the whole input is tokenised in ONE library call
// straight into the mapping at its final offset (blt_bpe_process_chunks pipelines its windows over
// the devices and writes each window's tokens in chunk order, pipeline.rs:153-192), then the file
// is cut to the bytes produced.  No host buffer and no write(2): the page-cache copy that bounded
// the windowed path (one inode lock, ~5.5 GB/s on tmpfs) becomes the runtime's device-to-host
// copies into pages the preallocation below already holds.  Returns 1 (nothing done) when the
// file cannot be sized or mapped, so the caller takes the windowed path.
struct OutMap {
    uint8_t* m = nullptr;   // shared mapping of the output file, `total` bytes
    size_t total = 0;
    bool sized = false;     // the file was ftruncate'd to total (undone when the mapping failed)
    bool registered = false;
};

// The output file sized to its bound and mapped, its first `est` bytes' pages allocated
// (preallocate) and mapped writable (MADV_POPULATE_WRITE, several threads): on a helper thread while
// the HIP runtime starts, so the device-to-host copies of the run land in pages that are already
// there.  (Page faults under the copies, one per 4 KiB page, were most of the CLI's tokenise phase.)
void map_output(int fd, size_t total, size_t est, OutMap* om);

// BLT_CLI_TIMING: a step's end, seconds since the first such stamp (stderr)
void tstamp(const char* what) {
    static const bool on = getenv("BLT_CLI_TIMING") != nullptr;
    if (!on) return;
    static timespec t0 = [] { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t; }();
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    fprintf(stderr, "blt timing: step: %s %.4f s\n", what,
            (double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec));
}

int run_mmap_direct(const Strategy& st, const uint8_t* in, size_t n, size_t cs, int fd, size_t head,
                    const uint8_t* head_bytes, const OutMap& om, std::vector<std::thread>& behind,
                    const std::string& span) {
    const size_t cap = st.kind == Strategy::kPassthrough ? n : 2 * n;
    const size_t total = head + cap;
    if (total == 0) return 0;
    if (!om.m || om.total != total) {
        if (om.sized) (void)ftruncate(fd, 0);
        return 1;
    }
    uint8_t* out = om.m;
    if (head) memcpy(out, head_bytes, head);
    size_t olen = 0;
    int rc = 0;
    if (n && st.kind == Strategy::kBpe) {
        rc = blt_bpe_process_chunks(st.h, in, n, cs, st.gpus, out + head, cap, &olen, nullptr);
    } else {
        // passthrough and basic are position-wise (tokenizer.rs:108-124, :129-137): pieces of 256 MiB
        constexpr size_t kPiece = size_t(256) << 20;
        for (size_t off = 0; off < n && !rc; off += kPiece) {
            const size_t len = std::min(kPiece, n - off);
            size_t w = 0;
            if (st.kind == Strategy::kPassthrough) {
                memcpy(out + head + olen, in + off, len);
                w = len;
            } else {
                rc = blt_basic_process_chunk(in + off, len, out + head + olen, cap - olen, &w);
            }
            olen += w;
        }
    }
    if (!rc) log_chunks(span, st.kind == Strategy::kBasic, 0, (n + cs - 1) / cs, n, cs);
    tstamp("tokens in the output mapping");
    for (auto& t : behind) t.join();   // (populate_behind: done with the mapping too)
    behind.clear();
    tstamp("helper threads joined");
    if (om.registered) (void)hipHostUnregister(om.m);
    munmap(om.m, total);
    tstamp("output unmapped");
    const std::string msg = rc ? last_error() : std::string();
    // the bytes produced (an error leaves the content token only, like a run that wrote no chunk)
    if (ftruncate(fd, (off_t)(head + (rc ? 0 : olen))) != 0 && !rc) return os_error(errno);
    tstamp("output truncated");
    if (rc) return set_error(rc, "%s", msg.c_str());
    return 0;
}

// Page allocation of the output file's first `bytes` ahead of the writes (FALLOC_FL_KEEP_SIZE: the
// file's size is unchanged), on a helper thread while the HIP runtime starts: on tmpfs most of a
// write's cost is allocating and zeroing pages (1 GiB: ~0.06 s to fallocate, then copies run ~2x
// faster, profiles/r03_tmpfs_write.txt).  Best effort: an error leaves the writes to allocate.
void preallocate(int fd, size_t bytes) {
    constexpr size_t kStep = size_t(64) << 20;
    for (size_t off = 0; off < bytes; off += kStep)
        if (fallocate(fd, FALLOC_FL_KEEP_SIZE, (off_t)off, (off_t)std::min(kStep, bytes - off)) != 0) return;
}

bool env_on(const char* name, bool dflt) {
    const char* v = getenv(name);
    return (v && *v) ? strcmp(v, "0") != 0 : dflt;
}

void map_output(int fd, size_t total, size_t est, OutMap* om) {
    if (ftruncate(fd, (off_t)total) != 0) return;
    om->sized = true;
    void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) return;
    om->m = static_cast<uint8_t*>(m);
    om->total = total;
    const size_t len = std::min(est, total);
    // (env: A/B runs) 0 fallocate only (the default), 1 fallocate then populate (MADV_POPULATE_WRITE,
    // BLT_OUT_THREADS threads), 2 populate only (it allocates too), with MADV_HUGEPAGE first when
    // BLT_OUT_HUGE is set (tmpfs huge pages where the host allows them; the GPU box's shmem THP is
    // "never").  Measured (profiles/r04_cli_phases.json): populating makes the device-to-host copies
    // 3x faster (tools/copy_probe.cpp: 0.139 -> 0.042 s per GiB), but the page-fault storm holds the
    // process's mmap lock while the HIP runtime starts on the other thread, and its start-up went
    // from 0.11-0.13 to 0.23 s: no net gain, so the writes fault their own pages.
    const char* pv = getenv("BLT_OUT_POPULATE");
    const int mode = (pv && *pv) ? atoi(pv) : 0;
    const char* tv = getenv("BLT_OUT_THREADS");
    const size_t nt = std::max<size_t>(1, std::min<size_t>(16, (tv && *tv) ? (size_t)atoi(tv) : 4));
    if (env_on("BLT_OUT_HUGE", false)) (void)madvise(m, total, MADV_HUGEPAGE);
    if (mode == 1 || mode == 0) preallocate(fd, len);
    if (mode >= 1) {
        // 2 MiB-aligned pieces over nt threads; best effort (older kernels: EINVAL, the copies fault)
        constexpr size_t kPiece = size_t(2) << 20;
        const size_t pieces = (len + kPiece - 1) / kPiece;
        auto part = [&](size_t t) {
            for (size_t i = t; i < pieces; i += nt) {
                const size_t off = i * kPiece;
                if (madvise(om->m + off, std::min(kPiece, len - off), MADV_POPULATE_WRITE) != 0) return;
            }
        };
        std::vector<std::thread> th;
        for (size_t t = 1; t < nt; ++t) th.emplace_back(part, t);
        part(0);
        for (auto& t : th) t.join();
    }
    // (env experiment) the whole mapping page-locked for the runtime's copies
    if (env_on("BLT_OUT_REGISTER", false))
        om->registered = hipHostRegister(om->m, total, hipHostRegisterDefault) == hipSuccess;
}

// (experiment, off by default) The output's first `est` bytes mapped writable
// (MADV_POPULATE_WRITE) by `nt` threads in 2 MiB pieces from the start, once the HIP runtime is up
// and while the tokeniser runs, so that the device-to-host copies would land in pages already
// mapped.  Done at start-up (map_output, mode 1), the same page-fault storm held the process's mmap
// lock against the runtime's own start-up (0.11-0.13 -> 0.23 s); behind it, it contends with the
// copies themselves (run()).  Best effort: a piece that fails stops that thread.
void populate_behind(const OutMap& om, size_t est, std::vector<std::thread>& th) {
    const char* tv = getenv("BLT_OUT_THREADS");
    const size_t nt = std::max<size_t>(1, std::min<size_t>(16, (tv && *tv) ? (size_t)atoi(tv) : 4));
    constexpr size_t kPiece = size_t(2) << 20;
    const size_t len = std::min(est, om.total);
    const size_t pieces = (len + kPiece - 1) / kPiece;
    uint8_t* m = om.m;
    for (size_t t = 0; t < nt; ++t)
        th.emplace_back([=] {
            for (size_t i = t; i < pieces; i += nt) {
                const size_t off = i * kPiece;
                if (madvise(m + off, std::min(kPiece, len - off), MADV_POPULATE_WRITE) != 0) return;
            }
        });
}

// Stream path (pipeline.rs:196-433): one read per chunk, at most `threads` chunks in flight, a
// worker pool tokenises (each call stages its chunk through the GPU; the handle is reentrant), a
// writer emits results in chunk order.  Any error stops reading and is returned.
int run_stream(const Strategy& st, int in_fd, size_t cs, size_t threads, Sink& sink, const std::string& span) {
    const bool dbg = blt_log::on(blt_log::kDebug, blt_log::kPipeline) || blt_log::on(blt_log::kDebug, blt_log::kTokenizer);
    const std::string sp_read = span + ":manage_task_spawning";
    threads = std::max<size_t>(1, threads);
    const size_t nworkers = std::min<size_t>(threads, 16);
    const size_t rd = std::min(cs, kStdinReadCap);
    RunStatus status;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<uint64_t, std::vector<uint8_t>>> jobs;
    std::map<uint64_t, std::vector<uint8_t>> results;
    size_t in_flight = 0;   // read, not yet written
    uint64_t n_read = 0, n_written = 0;
    bool eof = false, stop = false;

    std::vector<std::thread> pool;
    for (size_t w = 0; w < nworkers; ++w)
        pool.emplace_back([&] {
            for (;;) {
                std::pair<uint64_t, std::vector<uint8_t>> job;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return !jobs.empty() || eof || stop; });
                    if (jobs.empty() || stop) return;
                    job = std::move(jobs.front());
                    jobs.pop_front();
                }
                std::vector<uint8_t> out;
                if (dbg && st.kind == Strategy::kBasic && !job.second.empty()) {
                    const std::string sp = span + ":process_chunk_task{task_id=" + std::to_string(job.first) +
                                           "}:basic_tokenization_strategy_process";
                    blt_log::emit(blt_log::kDebug, sp.c_str(), "blt_core::tokenizer", "Converting %zu bytes to u16 tokens",
                                  job.second.size());
                }
                const int rc = st.chunk(job.second.data(), job.second.size(), out);
                std::lock_guard<std::mutex> lk(mu);
                if (dbg) blt_log::emit(blt_log::kDebug, span.c_str(), "blt_core::pipeline", "Received result for task task_id=%llu",
                                       (unsigned long long)job.first);
                if (rc) {
                    // (pipeline.rs:409: the error reaches the ordered writer; here the first error stops the run)
                    blt_log::emit(blt_log::kError, span.c_str(), "blt_core::pipeline",
                                  "Error in processed chunk: %s chunk_id=%llu", last_error().c_str(),
                                  (unsigned long long)job.first);
                    status.set(rc, last_error());
                    stop = true;
                } else {
                    results.emplace(job.first, std::move(out));
                }
                cv.notify_all();
            }
        });
    std::thread writer([&] {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return stop || results.count(n_written) || (eof && n_written == n_read); });
            if (stop) return;
            auto it = results.find(n_written);
            if (it == results.end()) return;   // eof and everything written
            std::vector<uint8_t> out = std::move(it->second);
            results.erase(it);
            lk.unlock();
            if (dbg) blt_log::emit(blt_log::kDebug, span.c_str(), "blt_core::pipeline", "Writing ordered chunk to output chunk_id=%llu bytes=%zu",
                                   (unsigned long long)n_written, out.size());
            const int rc = sink.write_all(out.data(), out.size());
            const std::string m = rc ? last_error() : std::string();
            lk.lock();
            if (rc) {
                status.set(rc, m);
                stop = true;
                cv.notify_all();
                return;
            }
            ++n_written;
            --in_flight;
            cv.notify_all();
        }
    });

    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return in_flight < threads || stop; });
            if (stop) break;
        }
        std::vector<uint8_t> chunk(rd);
        ssize_t r;
        do {
            r = ::read(in_fd, chunk.data(), rd);
        } while (r < 0 && errno == EINTR);
        std::lock_guard<std::mutex> lk(mu);
        if (r < 0) {
            status.set(os_error(errno), last_error());
            stop = true;
            cv.notify_all();
            break;
        }
        if (r == 0) {
            if (dbg) blt_log::emit(blt_log::kDebug, sp_read.c_str(), "blt_core::pipeline", "Input stream reached EOF");
            eof = true;
            cv.notify_all();
            break;
        }
        chunk.resize((size_t)r);
        if (dbg) blt_log::emit(blt_log::kDebug, sp_read.c_str(), "blt_core::pipeline", "Spawning chunk processing task task_id=%llu bytes=%zd",
                               (unsigned long long)n_read, r);
        jobs.emplace_back(n_read++, std::move(chunk));
        ++in_flight;
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        eof = true;
        cv.notify_all();
    }
    for (auto& t : pool) t.join();
    writer.join();
    if (status.rc) return set_error(status.rc, "%s", status.msg.c_str());
    return 0;
}

}  // namespace

// blt_host.cpp: device setup ahead of a blt_bpe_process_chunks call of this shape.
void blt_prewarm_chunks(const blt_bpe* h, uint64_t n, uint64_t cs, int n_gpus);

namespace {

int run(const blt_run_config* c) {
    if (!c) return set_error(BLT_E_INVALID_INPUT, "null config");
    if (c->chunk_size == 0) return set_error(BLT_E_INVALID_INPUT, "chunk_size must be > 0");
    if (c->content_token > 0xFFFFu) return set_error(BLT_E_INVALID_INPUT, "content token 0x%x is not a u16", c->content_token);
    // the run_tokenizer span (lib.rs:245: fields input, output as Option<PathBuf> Debug)
    auto opt = [](const char* path) { return path ? "Some(\"" + std::string(path) + "\")" : std::string("None"); };
    const std::string span = "run_tokenizer{input=" + opt(c->input_path) + " output=" + opt(c->output_path) + "}";
    const std::string span_pipe = span + ":run_pipeline";
    blt_log::emit(blt_log::kInfo, span.c_str(), "blt_core", "Starting tokenizer");
    Strategy st;
    if (c->passthrough) st.kind = Strategy::kPassthrough;   // lib.rs:272-274: passthrough wins
    else if (c->bpe) st.kind = Strategy::kBpe;
    else st.kind = Strategy::kBasic;
    blt_log::emit(blt_log::kInfo, span.c_str(), "blt_core",
                  st.kind == Strategy::kPassthrough ? "Using passthrough strategy (file copying without tokenization)."
                  : st.kind == Strategy::kBpe      ? "Using BPE tokenization strategy."
                                                    : "Using basic tokenization strategy (byte-to-u16 conversion).");
    blt_log::emit(blt_log::kInfo, span.c_str(), "blt_core", "Chunk size determined effective_chunk_size=%llu",
                  (unsigned long long)c->chunk_size);
    st.h = c->bpe;
    st.gpus = c->n_gpus;
    const size_t cs = (size_t)c->chunk_size;
    // HIP start-up and the first window's device setup run on a helper thread while the input is
    // mapped (BPE from a file): the device count, the handle's tables, staging buffers
    std::thread prewarm;
    auto gpu_count = [](int g) {
        if (g > 0) return g;
        int count = 0;
        return (hipGetDeviceCount(&count) == hipSuccess && count > 0) ? count : 1;
    };
    struct Join {
        std::thread& t;
        ~Join() { if (t.joinable()) t.join(); }
    } join_prewarm{prewarm};

    // setup_io (io_handler.rs:55-62): the input is opened and mapped first
    const bool timing = getenv("BLT_CLI_TIMING") != nullptr;
    timespec ts0;
    clock_gettime(CLOCK_MONOTONIC, &ts0);
    const uint8_t* map = nullptr;
    size_t n = 0;
    int in_populate = 2;
    if (c->input_path) {
        const int fd = ::open(c->input_path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) return os_error(errno);
        struct stat sb;
        if (fstat(fd, &sb) != 0) {
            const int e = errno;
            ::close(fd);
            return os_error(e);
        }
        n = (size_t)sb.st_size;
        if (st.kind == Strategy::kBpe && n && !getenv("BLT_NO_PREWARM")) {   // (env: A/B runs)
            const size_t per = std::max<size_t>(1, (size_t(256) << 20) / cs);   // run_mmap's window
            // the mapped-output path tokenises the whole input in one call (run_mmap_direct)
            const bool whole = c->output_path && !getenv("BLT_NO_DIRECT_OUTPUT");
            const uint64_t win = whole ? (uint64_t)n : std::min<uint64_t>(n, (uint64_t)per * cs);
            prewarm = std::thread([&st, &gpu_count, win, cs, timing, ts0] {
                auto since = [&ts0] {
                    timespec t;
                    clock_gettime(CLOCK_MONOTONIC, &t);
                    return (double)(t.tv_sec - ts0.tv_sec) + 1e-9 * (double)(t.tv_nsec - ts0.tv_nsec);
                };
                st.gpus = gpu_count(st.gpus);
                const double t_rt = timing ? since() : 0;
                blt_prewarm_chunks(st.h, win, cs, st.gpus);
                if (timing)
                    fprintf(stderr, "blt timing: prewarm: HIP runtime up at %.4f s, device tables and buffers at %.4f s\n",
                            t_rt, since());
            });
        }
        if (n) {
            // The file's pages are mapped in bulk, not page by page under the GPU copies, but only
            // once the HIP runtime is up (in_populate 2, the default: MADV_POPULATE_READ on helper
            // threads beside the tokeniser, run()): MAP_POPULATE here (1) held the process's mmap lock
            // while the runtime started on the prewarm thread, and the runtime came up at 0.12-0.28 s
            // instead of 0.06-0.10 s (profiles/r05_cli_phases.json).  (env: A/B runs) BLT_IN_POPULATE
            // 0 leaves the pages to the copies' own faults.
            const char* ipv = getenv("BLT_IN_POPULATE");
            in_populate = (ipv && *ipv) ? atoi(ipv) : 2;
            void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | (in_populate == 1 ? MAP_POPULATE : 0), fd, 0);
            if (m == MAP_FAILED) {
                const int e = errno;
                ::close(fd);
                return os_error(e);
            }
            madvise(m, n, MADV_SEQUENTIAL);
            map = static_cast<const uint8_t*>(m);
        }
        ::close(fd);
    }
    if (timing) {
        timespec ts1;
        clock_gettime(CLOCK_MONOTONIC, &ts1);
        fprintf(stderr, "blt timing: input open + mmap %.4f s\n",
                (double)(ts1.tv_sec - ts0.tv_sec) + 1e-9 * (double)(ts1.tv_nsec - ts0.tv_nsec));
    }
    struct Unmap {
        const uint8_t* p;
        size_t n;
        ~Unmap() {
            if (p) munmap(const_cast<uint8_t*>(p), n);
            tstamp("input unmapped");
        }
    } unmap{map, n};

    // setup_output_writer (io_handler.rs:70-78): File::create truncates; None is stdout.  Created
    // after the input (as the reference), but before the device is ready, so its pages can be
    // allocated meanwhile.
    Sink sink;
    int ofd = 1;
    if (c->output_path) {
        ofd = ::open(c->output_path, O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
        if (ofd < 0) {
            const int e = errno;
            if (prewarm.joinable()) prewarm.join();
            return os_error(e);
        }
        sink.fd = ofd;
        sink.positioned = true;
    }
    const size_t head = c->content_token ? 2 : 0;
    // the mapped-output path: a file input (fixed chunks) into a regular output file this run created
    bool direct = false;
    if (c->input_path && c->output_path && !getenv("BLT_NO_DIRECT_OUTPUT")) {
        struct stat ob;
        direct = fstat(ofd, &ob) == 0 && S_ISREG(ob.st_mode);
    }
    std::thread prealloc;
    OutMap om;
    if (direct && n) {
        // expected output: basic 2 bytes per byte; BPE about 1 (large merge maps: ~0.5 tokens per byte)
        const size_t est = head + (st.kind == Strategy::kBasic ? 2 * n : n);
        const size_t total = head + (st.kind == Strategy::kPassthrough ? n : 2 * n);
        prealloc = std::thread([ofd, total, est, &om] { map_output(ofd, total, est, &om); });
    }
    // (env experiment) the input mapping page-locked for the runtime's copies, beside the device setup
    bool in_registered = false;
    std::thread reg_in;
    if (map && st.kind == Strategy::kBpe && env_on("BLT_IN_REGISTER", false))
        reg_in = std::thread([map, n, &in_registered] {
            in_registered = hipHostRegister(const_cast<uint8_t*>(map), n, hipHostRegisterReadOnly) == hipSuccess;
        });
    if (prewarm.joinable()) prewarm.join();
    else if (st.kind == Strategy::kBpe) st.gpus = gpu_count(st.gpus);
    if (prealloc.joinable()) prealloc.join();
    if (reg_in.joinable()) reg_in.join();
    struct Unregister {
        const uint8_t* p;
        bool on;
        ~Unregister() { if (on) (void)hipHostUnregister(const_cast<uint8_t*>(p)); }
    } unregister{map, in_registered};
    if (timing) {
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        fprintf(stderr, "blt timing: device ready and output preallocated at %.4f s\n",
                (double)(t.tv_sec - ts0.tv_sec) + 1e-9 * (double)(t.tv_nsec - ts0.tv_nsec));
    }
    auto stamp = [&](const char* what) {
        if (!timing) return;
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        fprintf(stderr, "blt timing: %s at %.4f s\n", what,
                (double)(t.tv_sec - ts0.tv_sec) + 1e-9 * (double)(t.tv_nsec - ts0.tv_nsec));
    };
    stamp("output opened (truncated)");
    struct Close {
        int fd;
        ~Close() { if (fd > 2) ::close(fd); }
    } closer{c->output_path ? ofd : -1};

    int rc = 0;
    const uint8_t tok[2] = {(uint8_t)(c->content_token >> 8), (uint8_t)c->content_token};
    if (c->input_path)
        blt_log::emit(blt_log::kInfo, span_pipe.c_str(), "blt_core::pipeline", "Running pipeline in Mmap mode for file of size: %zu", n);
    else
        blt_log::emit(blt_log::kInfo, span_pipe.c_str(), "blt_core::pipeline", "Running pipeline in Stream mode for stdin");
    int drc = 1;
    std::vector<std::thread> behind;
    struct JoinAll {
        std::vector<std::thread>& v;
        ~JoinAll() { for (auto& t : v) if (t.joinable()) t.join(); }
    } join_behind{behind};
    if (map && in_populate == 2) {   // the input's pages on 4 threads, behind the runtime's start-up
        uint8_t* im = const_cast<uint8_t*>(map);
        constexpr size_t kPiece = size_t(2) << 20;
        const size_t pieces = (n + kPiece - 1) / kPiece;
        for (size_t t = 0; t < 4; ++t)
            behind.emplace_back([=] {
                for (size_t i = t; i < pieces; i += 4)
                    if (madvise(im + i * kPiece, std::min(kPiece, n - i * kPiece), MADV_POPULATE_READ) != 0) return;
            });
    }
    if (direct) {
        // (env experiment, off: BLT_OUT_BEHIND=1) the output's pages mapped behind the start-up.
        // Measured (profiles/r05_cli_phases.json): device ready -> chunks written 0.29-0.35 s with
        // it, 0.24-0.28 s without: the populating threads and the runtime's copies into the same
        // mapping contend, so the copies fault their own pages.
        const char* pv = getenv("BLT_OUT_POPULATE");
        if (om.m && !(pv && *pv && atoi(pv) != 0) && env_on("BLT_OUT_BEHIND", false))
            populate_behind(om, head + (st.kind == Strategy::kBasic ? 2 * n : n), behind);
        drc = run_mmap_direct(st, map, n, cs, ofd, head, tok, om, behind, span_pipe);
    }
    if (drc <= 0) {
        rc = drc;
    } else {
        if (c->content_token) rc = sink.write_all(tok, 2);   // prepend_content_type_token (lib.rs:284-293)
        if (!rc) {
            if (c->input_path) rc = run_mmap(st, map, n, cs, sink, span_pipe);
            else rc = run_stream(st, 0, cs, (size_t)c->threads, sink, span_pipe);
        }
    }
    stamp("chunks written");
    if (!rc && c->output_path) {
        closer.fd = -1;
        if (::close(ofd) != 0) rc = os_error(errno);
    }
    stamp("output closed");
    if (!rc) blt_log::emit(blt_log::kInfo, span.c_str(), "blt_core", "Tokenizer run completed successfully");
    return rc;
}

}  // namespace

extern "C" int blt_run_tokenizer(const blt_run_config* cfg) {
    try {
        return run(cfg);
    } catch (const std::bad_alloc&) {
        return set_error(BLT_E_NOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return set_error(BLT_E_IO, "%s", e.what());
    }
}
