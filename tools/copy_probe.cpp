// Host<->device copy rates from the kinds of host memory the CLI's direct path uses (round 4):
// anonymous memory, a private read-only mapping of a tmpfs file (the input), a shared writable
// mapping of a tmpfs file (the output), populated or not.  One 1 GiB hipMemcpyAsync per case (and
// in 64 MiB pieces), timed on the host around a stream synchronize.
//   hipcc -O2 --offload-arch=gfx950 tools/copy_probe.cpp -o build/copy_probe && build/copy_probe
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static const size_t kN = size_t(1) << 30;

static double copy(void* dst, const void* src, size_t piece, hipMemcpyKind kind, hipStream_t s) {
    const double t0 = now();
    for (size_t off = 0; off < kN; off += piece)
        CK(hipMemcpyAsync((char*)dst + off, (const char*)src + off, piece, kind, s));
    CK(hipStreamSynchronize(s));
    return now() - t0;
}

static void report(const char* what, double t) { printf("%-58s %7.4f s  %6.2f GB/s\n", what, t, kN / t / 1e9); }

int main() {
    const char* dir = getenv("PROBE_DIR") ? getenv("PROBE_DIR") : "/dev/shm";
    char inpath[256], outpath[256];
    snprintf(inpath, sizeof inpath, "%s/copy_probe_in_%d", dir, (int)getpid());
    snprintf(outpath, sizeof outpath, "%s/copy_probe_out_%d", dir, (int)getpid());
    double t = now();
    CK(hipFree(nullptr));
    report("HIP init", now() - t);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void* d = nullptr;
    CK(hipMalloc(&d, kN));

    // input file
    {
        int fd = open(inpath, O_RDWR | O_CREAT | O_TRUNC, 0600);
        char* buf = (char*)malloc(1 << 20);
        memset(buf, 'a', 1 << 20);
        for (size_t off = 0; off < kN; off += 1 << 20) if (write(fd, buf, 1 << 20) != (1 << 20)) return 1;
        free(buf);
        close(fd);
    }
    char* anon = (char*)malloc(kN);
    memset(anon, 1, kN);
    for (int rep = 0; rep < 2; ++rep) {
        report("H2D anonymous (touched), 1 piece", copy(d, anon, kN, hipMemcpyHostToDevice, s));
        report("H2D anonymous (touched), 64 MiB pieces", copy(d, anon, 64 << 20, hipMemcpyHostToDevice, s));
        report("D2H anonymous (touched), 1 piece", copy(anon, d, kN, hipMemcpyDeviceToHost, s));
        report("D2H anonymous (touched), 64 MiB pieces", copy(anon, d, 64 << 20, hipMemcpyDeviceToHost, s));
    }
    free(anon);
    {
        int fd = open(inpath, O_RDONLY);
        t = now();
        void* m = mmap(nullptr, kN, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
        report("  mmap private read-only MAP_POPULATE", now() - t);
        close(fd);
        report("H2D private read-only file mapping, 1 piece", copy(d, m, kN, hipMemcpyHostToDevice, s));
        report("H2D private read-only file mapping, again", copy(d, m, kN, hipMemcpyHostToDevice, s));
        report("H2D private read-only file mapping, 64 MiB pieces", copy(d, m, 64 << 20, hipMemcpyHostToDevice, s));
        munmap(m, kN);
        fd = open(inpath, O_RDONLY);
        m = mmap(nullptr, kN, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
        close(fd);
        report("H2D shared read-only file mapping, 64 MiB pieces", copy(d, m, 64 << 20, hipMemcpyHostToDevice, s));
        munmap(m, kN);
    }
    for (int mode = 0; mode < 3; ++mode) {
        int fd = open(outpath, O_RDWR | O_CREAT | O_TRUNC, 0600);
        if (ftruncate(fd, (off_t)kN)) return 1;
        t = now();
        if (mode >= 1) for (size_t off = 0; off < kN; off += 64 << 20) fallocate(fd, FALLOC_FL_KEEP_SIZE, off, 64 << 20);
        const double tf = now() - t;
        void* m = mmap(nullptr, kN, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        t = now();
        int prc = 0;
        if (mode == 2) prc = madvise(m, kN, 23 /* MADV_POPULATE_WRITE */);
        const double tp = now() - t;
        char what[128];
        snprintf(what, sizeof what, "  output: fallocate %.4f s, populate %.4f s (rc %d)", tf, tp, prc);
        report(what, tf + tp);
        const char* names[3] = {"D2H shared file mapping, fresh, 64 MiB pieces", "D2H shared file mapping, fallocated, 64 MiB pieces",
                                "D2H shared file mapping, populated, 64 MiB pieces"};
        report(names[mode], copy(m, d, 64 << 20, hipMemcpyDeviceToHost, s));
        report("  same mapping again", copy(m, d, 64 << 20, hipMemcpyDeviceToHost, s));
        t = now();
        munmap(m, kN);
        close(fd);
        unlink(outpath);
        report("  munmap + unlink", now() - t);
    }
    unlink(inpath);
    CK(hipFree(d));
    return 0;
}
