// threads_test.cpp -- TEST PROGRAM: distinct drop-in resizer objects used concurrently from
// several host threads (include/iqo_hip.h "Threading": a plan from one thread at a time, distinct
// plans independent; the host path borrows one pooled staging set per call, abi.hip).
//
//   threads_test OUT_DIR THREADS ROUNDS
//
// Jobs (one per thread, cycling over Lanczos / Area / Linear shapes, each with its own input):
// every job is first run alone; then all threads run their jobs at once, ROUNDS times, each
// thread constructing a fresh object per round (as the reference benchmark does,
// benchmark.cpp:215-226) and comparing with its solo output.  Exit status 0 = every concurrent
// output byte-identical to the solo one; each job's solo output and input go to OUT_DIR for the
// Python test to check against the Generic oracle.
#include <iqo_hip.h>
#include <libiqo/iqo.hpp>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Job {
    int method;  // 0 lanczos, 1 area, 2 linear
    unsigned degree;
    size_t sw, sh, dw, dh;
    std::vector<unsigned char> src, solo;
};

void run(const Job &j, unsigned char *dst)
{
    if (j.method == 0) {
        iqo::LanczosResizer r(j.degree, j.sw, j.sh, j.dw, j.dh);
        r.resize(j.sw, j.src.data(), j.dw, dst);
    } else if (j.method == 1) {
        iqo::AreaResizer r(j.sw, j.sh, j.dw, j.dh);
        r.resize(j.sw, j.src.data(), j.dw, dst);
    } else {
        iqo::LinearResizer r(j.sw, j.sh, j.dw, j.dh);
        r.resize(j.sw, j.src.data(), j.dw, dst);
    }
}

} // namespace

int main(int argc, char **argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: threads_test OUT_DIR THREADS ROUNDS\n");
        return 2;
    }
    const std::string out = argv[1];
    const int nThreads = std::atoi(argv[2]), rounds = std::atoi(argv[3]);
    static const struct { int m; unsigned d; size_t sw, sh, dw, dh; } shapes[] = {
        {0, 3, 1920, 1080, 960, 540}, {1, 0, 1920, 1080, 480, 270}, {2, 0, 960, 540, 1920, 1080},
        {0, 2, 640, 480, 320, 240},   {0, 3, 1280, 720, 1920, 1080}, {1, 0, 1000, 600, 640, 400},
    };
    std::vector<Job> jobs(static_cast<size_t>(nThreads));
    for (int t = 0; t < nThreads; ++t) {
        const auto &s = shapes[t % 6];
        Job &j = jobs[static_cast<size_t>(t)];
        j.method = s.m;
        j.degree = s.d;
        j.sw = s.sw;
        j.sh = s.sh;
        j.dw = s.dw;
        j.dh = s.dh;
        j.src.resize(s.sw * s.sh);
        unsigned x = 2463534242u + 977u * static_cast<unsigned>(t);
        for (auto &b : j.src) {  // xorshift32
            x ^= x << 13;
            x ^= x >> 17;
            x ^= x << 5;
            b = static_cast<unsigned char>(x >> 24);
        }
        j.solo.assign(s.dw * s.dh, 0);
        run(j, j.solo.data());
        char name[512];
        std::snprintf(name, sizeof name, "%s/job%02d_%d_%u_%zux%zu_%zux%zu", out.c_str(), t, s.m, s.d, s.sw, s.sh,
                      s.dw, s.dh);
        FILE *f = std::fopen((std::string(name) + ".src").c_str(), "wb");
        FILE *g = std::fopen((std::string(name) + ".dst").c_str(), "wb");
        if (!f || !g)
            return 3;
        std::fwrite(j.src.data(), 1, j.src.size(), f);
        std::fwrite(j.solo.data(), 1, j.solo.size(), g);
        std::fclose(f);
        std::fclose(g);
    }
    std::atomic<int> bad(0);
    for (int r = 0; r < rounds; ++r) {
        std::vector<std::thread> th;
        for (int t = 0; t < nThreads; ++t)
            th.emplace_back([&, t] {
                const Job &j = jobs[static_cast<size_t>(t)];
                std::vector<unsigned char> dst(j.dw * j.dh, 0x5a);
                run(j, dst.data());
                if (std::memcmp(dst.data(), j.solo.data(), dst.size()) != 0)
                    ++bad;
            });
        for (auto &x : th)
            x.join();
    }
    int onHip = 0, onCpu = 0;
    iqo_dropin_backend_counts(&onHip, &onCpu);
    std::printf("threads %d rounds %d mismatches %d\n", nThreads, rounds, bad.load());
    std::printf("backend: hip %d cpu %d\n", onHip, onCpu);
    return bad.load() ? 1 : 0;
}
