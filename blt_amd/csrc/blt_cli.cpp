// blt — command-line drop-in for jtrefon/blt's `blt` binary (src/main.rs:8-60), over the C ABI
// of libblt_bpe.so (include/blt_bpe.h).  Same flags, same defaults, same output bytes:
//
//   -i/--input FILE|-      input file (mmap) or stdin            (main.rs:11-17, io_handler.rs:55-62)
//   -o/--output FILE|-     output file or stdout                 (main.rs:19-25, io_handler.rs:70-78)
//   --merges FILE          BPE merges file -> BpeStrategy        (main.rs:27-32, lib.rs:271-282)
//   --passthrough          copy input unchanged                  (main.rs:34-35, tokenizer.rs:129-137)
//   --type text|audio|bin|video   prepend 0xFF01..0xFF04 (BE)   (main.rs:37-38, lib.rs:96-107, :284-293)
//   --threads N            chunks in flight (0 -> 1; default: all cores)   (utils.rs:83-101)
//   --memcap PERCENT       RAM share for the automatic chunk size (default 80)  (lib.rs:172)
//   --chunksize SIZE       "4MB", "256KB", raw bytes; clamped to [256 KiB, 128 MiB] (chunking.rs:26-31)
// plus one MI355X option:
//   --gpus N               devices the file path shards its chunks over (default: all visible)
//
// Tokenising runs on the GPU only (there is no CPU fallback: without a device the BPE and basic
// paths fail with the library's error).  Two input paths, as the reference (pipeline.rs:22-51):
//  * a file is mapped and cut into fixed chunk-size chunks (pipeline.rs:73-81); windows of whole
//    chunks go to blt_bpe_process_chunks / blt_basic_process_chunk while the previous window is
//    written, so the output is the chunk outputs concatenated in order (pipeline.rs:153-192);
//  * stdin is read one read() call per chunk of at most chunk-size bytes (pipeline.rs:303-318:
//    a short read makes a short chunk, exactly as tokio's read does), up to --threads chunks are
//    tokenised concurrently and written in chunk order.
// Errors: configuration errors print "Error: <message>" and exit 1 (main's io::Result); pipeline
// errors print "Error running tokenizer: <message>" and exit 1 (main.rs:99-102).
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/blt_bpe.h"

namespace {

struct Args {
    std::string input, output, merges;
    bool has_input = false, has_output = false, has_merges = false, passthrough = false;
    int content_token = -1;
    bool has_threads = false;
    uint64_t threads = 0;
    uint32_t memcap = 80;
    bool has_chunksize = false;
    std::string chunksize;
    int gpus = 0;   // 0: all visible
};

[[noreturn]] void usage(FILE* f, int code) {
    fprintf(f,
            "Usage: blt [OPTIONS]\n\n"
            "Options:\n"
            "  -i, --input <FILE>         Input file path (or - for stdin)\n"
            "  -o, --output <FILE>        Output file path (or - for stdout)\n"
            "      --merges <FILE>        BPE merges file for advanced tokenization\n"
            "      --passthrough          Use passthrough mode (copy file without tokenization)\n"
            "      --type <TYPE>          Prepend content-type token [possible values: text, audio, bin, video]\n"
            "      --threads <NUM>        Override worker count (default: auto based on cores)\n"
            "      --memcap <PERCENT>     Max RAM usage fraction (e.g., 70 for 70%%)\n"
            "      --chunksize <SIZE>     Min/Max chunk size (e.g. 4MB, 256KB).\n"
            "      --gpus <NUM>           GPUs the file path shards its chunks over (default: all)\n"
            "  -h, --help                 Print help\n"
            "  -V, --version              Print version\n");
    exit(code);
}

[[noreturn]] void arg_error(const char* fmt, const char* a) {
    fprintf(stderr, "error: ");
    fprintf(stderr, fmt, a);
    fprintf(stderr, "\n\nFor more information, try '--help'.\n");
    exit(2);   // clap's usage-error exit code
}

bool parse_u64(const char* s, uint64_t* v) {
    if (!*s) return false;
    char* end = nullptr;
    errno = 0;
    unsigned long long x = strtoull(s, &end, 10);
    if (errno || *end || s[0] == '-' || s[0] == '+') return false;
    *v = x;
    return true;
}

Args parse_args(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i], val;
        bool has_val = false;
        const size_t eq = k.find('=');
        if (k.rfind("--", 0) == 0 && eq != std::string::npos) {
            val = k.substr(eq + 1);
            k = k.substr(0, eq);
            has_val = true;
        }
        auto take = [&](const char* name) -> std::string {
            if (has_val) return val;
            if (i + 1 >= argc) arg_error("a value is required for '%s' but none was supplied", name);
            return argv[++i];
        };
        if (k == "-h" || k == "--help") usage(stdout, 0);
        if (k == "-V" || k == "--version") {
            printf("%s\n", blt_version());
            exit(0);
        }
        if (k == "-i" || k == "--input") {
            a.input = take("--input <FILE>");
            a.has_input = true;
        } else if (k == "-o" || k == "--output") {
            a.output = take("--output <FILE>");
            a.has_output = true;
        } else if (k == "--merges") {
            a.merges = take("--merges <FILE>");
            a.has_merges = true;
        } else if (k == "--passthrough") {
            a.passthrough = true;
        } else if (k == "--type") {
            const std::string t = take("--type <TYPE>");
            static const char* names[] = {"text", "audio", "bin", "video"};
            a.content_token = -1;
            for (int j = 0; j < 4; ++j)
                if (t == names[j]) a.content_token = 0xFF01 + j;   // lib.rs:96-107
            if (a.content_token < 0) arg_error("invalid value '%s' for '--type <TYPE>'", t.c_str());
        } else if (k == "--threads") {
            const std::string t = take("--threads <NUM>");
            if (!parse_u64(t.c_str(), &a.threads)) arg_error("invalid value '%s' for '--threads <NUM>'", t.c_str());
            a.has_threads = true;
        } else if (k == "--memcap") {
            const std::string t = take("--memcap <PERCENT>");
            uint64_t m = 0;
            if (!parse_u64(t.c_str(), &m) || m > 255) arg_error("invalid value '%s' for '--memcap <PERCENT>'", t.c_str());
            a.memcap = (uint32_t)m;   // u8 in the reference
        } else if (k == "--chunksize") {
            a.chunksize = take("--chunksize <SIZE>");
            a.has_chunksize = true;
        } else if (k == "--gpus") {
            const std::string t = take("--gpus <NUM>");
            uint64_t g = 0;
            if (!parse_u64(t.c_str(), &g) || g > 64) arg_error("invalid value '%s' for '--gpus <NUM>'", t.c_str());
            a.gpus = (int)g;
        } else {
            arg_error("unexpected argument '%s' found", argv[i]);
        }
    }
    // clap treats "-" as a path; the reference then opens a file named "-".  Here "-" means the
    // standard stream, as the help text promises.
    if (a.has_input && a.input == "-") a.has_input = false;
    if (a.has_output && a.output == "-") a.has_output = false;
    return a;
}

[[noreturn]] void config_error(const std::string& msg) {
    fprintf(stderr, "Error: %s\n", msg.c_str());
    exit(1);
}

[[noreturn]] void run_error(const std::string& msg) {
    fprintf(stderr, "Error running tokenizer: %s\n", msg.c_str());
    exit(1);
}

std::string lib_error(int rc) {
    const char* m = blt_last_error();
    return (m && *m) ? std::string(m) : ("error " + std::to_string(rc));
}

// Ordered sink over a file descriptor; write_all retries short writes.
struct Sink {
    int fd;
    bool regular = false;   // a regular file: large writes split over threads with pwrite
    off_t pos = 0;
    static void put(int fd, const uint8_t* p, size_t n, off_t at, bool positioned) {
        while (n) {
            const ssize_t w = positioned ? ::pwrite(fd, p, n, at) : ::write(fd, p, n);
            if (w < 0) {
                if (errno == EINTR) continue;
                run_error(std::string("write failed: ") + strerror(errno));
            }
            p += w;
            n -= (size_t)w;
            at += w;
        }
    }
    void write_all(const uint8_t* p, size_t n) {
        constexpr size_t kPart = size_t(32) << 20;
        if (!regular || n < 2 * kPart) {
            put(fd, p, n, pos, regular);
            pos += (off_t)n;
            return;
        }
        // page-cache copies of one big write scale with threads (the write order on disk is the
        // page cache's business; the file's bytes are the same)
        const size_t parts = std::min<size_t>(8, n / kPart);
        const size_t each = (n / parts + 4095) & ~size_t(4095);
        std::vector<std::thread> th;
        for (size_t i = 1; i < parts; ++i) {
            const size_t b = i * each;
            if (b >= n) break;
            th.emplace_back([=] { put(fd, p + b, std::min(each, n - b), pos + (off_t)b, true); });
        }
        put(fd, p, std::min(each, n), pos, true);
        for (auto& t : th) t.join();
        pos += (off_t)n;
    }
};

// An output buffer that is never zero-filled (a std::vector resize would clear a window's worth
// of bytes the GPU then overwrites) and keeps its pages between windows.
struct Buf {
    std::unique_ptr<uint8_t[]> p;
    size_t cap = 0, len = 0;
    void reserve(size_t n) {
        if (cap >= n) return;
        p.reset(new uint8_t[n]);
        cap = n;
    }
};

// The per-chunk transform for one strategy (tokenizer.rs:21-31): output appended to `out`.
struct Strategy {
    enum Kind { kPassthrough, kBpe, kBasic } kind;
    blt_bpe* h = nullptr;
    int gpus = 1;

    void chunk(const uint8_t* in, size_t n, std::vector<uint8_t>& out) const {
        out.clear();
        if (n == 0) return;
        if (kind == kPassthrough) {
            out.assign(in, in + n);
            return;
        }
        out.resize(2 * n);
        size_t olen = 0;
        const int rc = kind == kBpe ? blt_bpe_process_chunk(h, in, n, out.data(), out.size(), &olen)
                                    : blt_basic_process_chunk(in, n, out.data(), out.size(), &olen);
        if (rc) run_error(lib_error(rc));
        out.resize(olen);
    }

    // A window of whole chunks (the last may be short): outputs concatenated in chunk order.
    // Passthrough and basic are position-wise, so the window's output is the chunk outputs
    // concatenated (tokenizer.rs:108-124, :129-137).
    void window(const uint8_t* in, size_t n, size_t cs, Buf& out) const {
        out.len = 0;
        if (n == 0) return;
        if (kind == kPassthrough) {
            out.reserve(n);
            memcpy(out.p.get(), in, n);
            out.len = n;
            return;
        }
        out.reserve(2 * n);
        size_t olen = 0;
        const int rc = kind == kBpe ? blt_bpe_process_chunks(h, in, n, cs, gpus, out.p.get(), out.cap, &olen, nullptr)
                                    : blt_basic_process_chunk(in, n, out.p.get(), out.cap, &olen);
        if (rc) run_error(lib_error(rc));
        out.len = olen;
    }
};

// File path: mmap, windows of whole chunks, window k+1 tokenised while window k is written.
void run_mmap(const Strategy& st, const std::string& path, size_t cs, Sink& sink) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) config_error(path + ": " + strerror(errno));
    struct stat sb;
    if (fstat(fd, &sb) != 0) config_error(path + ": " + strerror(errno));
    const size_t n = (size_t)sb.st_size;
    if (n == 0) {
        ::close(fd);
        return;
    }
    // MAP_POPULATE maps the whole file up front (fault-around in bulk, no per-page faults while
    // the GPU copies read it)
    const bool timing = getenv("BLT_CLI_TIMING") != nullptr;   // phase times on stderr (tools/cli_rate.py)
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_map = now();
    void* map = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (map == MAP_FAILED) config_error(path + ": mmap failed: " + strerror(errno));
    ::close(fd);
    const uint8_t* in = static_cast<const uint8_t*>(map);
    madvise(map, n, MADV_SEQUENTIAL);

    // windows of whole chunks, about 256 MiB of input each
    const size_t per = std::max<size_t>(1, (size_t(256) << 20) / cs);
    const size_t win = per * cs;
    Buf buf[2];
    std::thread writer;
    double t_tok = 0, t_wait = 0, t0 = now();
    const double t_mapped = t0;
    for (size_t off = 0, k = 0; off < n; off += win, ++k) {
        const size_t len = std::min(win, n - off);
        Buf& out = buf[k & 1];
        st.window(in + off, len, cs, out);
        const double t1 = now();
        if (writer.joinable()) writer.join();   // window k-1 written: its buffer is free
        const double t2 = now();
        t_tok += t1 - t0;
        t_wait += t2 - t1;
        t0 = t2;
        writer = std::thread([&sink, &out] { sink.write_all(out.p.get(), out.len); });
    }
    if (writer.joinable()) writer.join();
    if (timing)
        fprintf(stderr, "blt timing: map %.4f s, tokenise %.4f s, writer wait %.4f s, last write %.4f s\n",
                t_mapped - t_map, t_tok, t_wait, now() - t0);
    munmap(map, n);
}

// Stdin path: one read() per chunk (pipeline.rs:303-318), at most --threads chunks in flight,
// written in chunk order (pipeline.rs:330-370).  A fixed pool tokenises (each call stages its
// chunk through the GPU; the handle is reentrant), a writer thread emits results in order.
void run_stream(const Strategy& st, size_t cs, size_t threads, Sink& sink) {
    const size_t nworkers = std::max<size_t>(1, std::min<size_t>(threads, 8));
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<uint64_t, std::vector<uint8_t>>> jobs;
    std::map<uint64_t, std::vector<uint8_t>> results;
    size_t in_flight = 0;   // read, not yet written
    uint64_t n_read = 0, n_written = 0;
    bool eof = false;

    std::vector<std::thread> pool;
    for (size_t w = 0; w < nworkers; ++w)
        pool.emplace_back([&] {
            for (;;) {
                std::pair<uint64_t, std::vector<uint8_t>> job;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return !jobs.empty() || eof; });
                    if (jobs.empty()) return;
                    job = std::move(jobs.front());
                    jobs.pop_front();
                }
                std::vector<uint8_t> out;
                st.chunk(job.second.data(), job.second.size(), out);
                std::lock_guard<std::mutex> lk(mu);
                results.emplace(job.first, std::move(out));
                cv.notify_all();
            }
        });
    std::thread writer([&] {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return results.count(n_written) || (eof && n_written == n_read); });
            auto it = results.find(n_written);
            if (it == results.end()) return;   // eof and everything written
            std::vector<uint8_t> out = std::move(it->second);
            results.erase(it);
            lk.unlock();
            sink.write_all(out.data(), out.size());
            lk.lock();
            ++n_written;
            --in_flight;
            cv.notify_all();
        }
    });

    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return in_flight < threads; });
        }
        std::vector<uint8_t> chunk(cs);
        ssize_t r;
        do {
            r = ::read(0, chunk.data(), cs);
        } while (r < 0 && errno == EINTR);
        if (r < 0) run_error(std::string("read failed: ") + strerror(errno));
        std::lock_guard<std::mutex> lk(mu);
        if (r == 0) {
            eof = true;
            cv.notify_all();
            break;
        }
        chunk.resize((size_t)r);
        jobs.emplace_back(n_read++, std::move(chunk));
        ++in_flight;
        cv.notify_all();
    }
    for (auto& t : pool) t.join();
    writer.join();
}

}  // namespace

static double mono_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const double t_main = mono_now();
    const Args a = parse_args(argc, argv);

    // CoreConfig::new_from_cli (lib.rs:149-174): threads, chunk size string, merges file
    const uint64_t threads = blt_determine_thread_count(a.has_threads ? 1 : 0, a.threads);
    uint64_t cli_cs = 0;
    if (a.has_chunksize) {
        const int rc = blt_parse_chunk_size(a.chunksize.c_str(), &cli_cs);
        if (rc) config_error(lib_error(rc));
    }
    Strategy st;
    st.gpus = a.gpus;
    if (a.passthrough) {
        st.kind = Strategy::kPassthrough;   // lib.rs:272-274: passthrough wins over merges
    } else if (a.has_merges) {
        st.kind = Strategy::kBpe;
        const int rc = blt_bpe_create_from_file(a.merges.c_str(), &st.h);
        if (rc) config_error(lib_error(rc));   // "Failed to load BPE merges: ..." (lib.rs:195-201)
    } else {
        st.kind = Strategy::kBasic;
    }
    if (a.passthrough && a.has_merges) {
        // the reference still loads (and validates) the merges file before picking passthrough
        blt_bpe* tmp = nullptr;
        const int rc = blt_bpe_create_from_file(a.merges.c_str(), &tmp);
        if (rc) config_error(lib_error(rc));   // "Failed to load BPE merges: ..." (lib.rs:195-201)
        blt_bpe_destroy(tmp);
    }
    if (st.kind == Strategy::kBpe && a.gpus == 0) st.gpus = 64;   // all visible devices
    const uint64_t cs = blt_effective_chunk_size(a.has_chunksize ? 1 : 0, cli_cs, threads, a.memcap);

    // setup_io (io_handler.rs:55-79): the output file is created before any input is read
    int ofd = 1;
    if (a.has_output) {
        ofd = ::open(a.output.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (ofd < 0) config_error(a.output + ": " + strerror(errno));
    }
    if (a.has_input && ::access(a.input.c_str(), R_OK) != 0) config_error(a.input + ": " + strerror(errno));
    Sink sink{ofd};
    {
        struct stat ob;
        sink.regular = fstat(ofd, &ob) == 0 && S_ISREG(ob.st_mode) && lseek(ofd, 0, SEEK_CUR) == 0;
    }
    if (a.content_token >= 0) {   // prepend_content_type_token (lib.rs:284-293)
        const uint8_t t[2] = {(uint8_t)(a.content_token >> 8), (uint8_t)a.content_token};
        sink.write_all(t, 2);
    }
    const double t_run = mono_now();
    if (a.has_input)
        run_mmap(st, a.input, (size_t)cs, sink);
    else
        run_stream(st, (size_t)cs, (size_t)threads, sink);
    const double t_done = mono_now();
    if (st.h) blt_bpe_destroy(st.h);
    if (getenv("BLT_CLI_TIMING"))
        fprintf(stderr, "blt timing: main at %.4f (monotonic), setup %.4f s, run %.4f s, teardown from %.4f\n", t_main,
                t_run - t_main, t_done - t_run, t_done);
    if (a.has_output && ::close(ofd) != 0) run_error(std::string("close failed: ") + strerror(errno));
    // Every byte is written with write()/pwrite() and the output is closed: leave without the
    // HIP runtime's exit-time teardown of the device contexts and pinned buffers (~0.4 s).
    fflush(nullptr);
    _exit(0);
}
