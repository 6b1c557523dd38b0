// iqo_benchmark -- command-line benchmark with the reference's interface
// (benchmark/benchmark.cpp:882-1036: `-m method -iw W -ih H -ow w -oh h`), running the drop-in
// iqo::*Resizer classes of this library (MI355X backend).
//
// Like the reference it resizes a YUV420 frame per cycle (Y at pxScale 1, U and V at half size;
// Lanczos chroma at pxScale 2, :206-229), constructs the resizers INSIDE the timed region, fills
// planes with std::mt19937(0) + uniform_int_distribution<int>(0,255) (:51-59) and prints the
// minimum ms/cycle over the cycles.  Extra flags (not in the reference):
//   -cycles N    number of cycles (default 256, as the reference)
//   -check FILE  write the Y-plane output to FILE (raw U8, stride = width) for parity checks
//   -reuse 1     construct the resizers once, outside the timed region
#include <iqo_hip.h>
#include <libiqo/iqo.hpp>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

namespace {

std::map<std::string, std::string> parse(int argc, char **argv)
{
    std::map<std::string, std::string> a;
    for (int i = 1; i < argc; ++i) {
        if (argv[i][0] == '-' && i + 1 < argc) {
            a[argv[i] + 1] = argv[i + 1];
            ++i;
        } else {
            a[argv[i]] = "true";
        }
    }
    return a;
}

void fill(std::vector<uint8_t> &v, size_t off, size_t n)
{
    std::mt19937 gen(0);
    std::uniform_int_distribution<int> dist(0, 255);
    for (size_t i = 0; i < n; ++i)
        v[off + i] = static_cast<uint8_t>(dist(gen));
}

struct Planes {
    size_t w, h, st;  // luma size and stride (stride of chroma = st/2)
    std::vector<uint8_t> buf;
    size_t y() const { return 0; }
    size_t u() const { return st * ((h + 1) & ~size_t(1)); }
    size_t v() const { return u() + (st / 2) * ((h + 1) / 2); }
};

} // namespace

int main(int argc, char **argv)
{
    std::map<std::string, std::string> a = parse(argc, argv);
    std::string method = a["m"];
    long iw = std::atol(a["iw"].c_str()), ih = std::atol(a["ih"].c_str());
    long ow = std::atol(a["ow"].c_str()), oh = std::atol(a["oh"].c_str());
    int cycles = a.count("cycles") ? std::atoi(a["cycles"].c_str()) : 256;
    bool reuse = a.count("reuse") && a["reuse"] != "0";
    if (!iw || !ih || !ow || !oh || cycles < 1) {
        std::printf("usage: iqo_benchmark -m method -iw in_width -ih in_height -ow out_width -oh out_height"
                    " [-cycles N] [-check out.raw] [-reuse 1]\nmethod: area | linear | lanczos[1-9]\n");
        return EINVAL;
    }
    int degree = 2;
    if (method.size() == 8 && method.compare(0, 7, "lanczos") == 0) {
        degree = method[7] - '0';
        if (degree < 1 || degree > 9) {
            std::printf("invalid method: %s\n", method.c_str());
            return EINVAL;
        }
        method = "lanczos";
    }
    if (method != "lanczos" && method != "area" && method != "linear") {
        std::printf("invalid method: %s\n", method.c_str());
        return EINVAL;
    }
    Planes s, d;
    s.w = iw;
    s.h = ih;
    s.st = iw + iw % 2;  // reference: strides rounded up to even (:921-930)
    d.w = ow;
    d.h = oh;
    d.st = ow + ow % 2;
    s.buf.assign(s.v() + (s.st / 2) * ((s.h + 1) / 2), 0);
    d.buf.assign(d.v() + (d.st / 2) * ((d.h + 1) / 2), 0);
    fill(s.buf, s.y(), s.st * s.h);
    fill(s.buf, s.u(), (s.st / 2) * (s.h / 2));
    fill(s.buf, s.v(), (s.st / 2) * (s.h / 2));

    std::printf("method: %s\n", method.c_str());
    if (method == "lanczos")
        std::printf("quality\n  degree: %d\n", degree);
    std::printf("backend\n  libiqo_amd (MI355X gfx950 HIP)\ninput\n    size: %ldx%ld\n  stride: %zu\noutput\n"
                "    size: %ldx%ld\n  stride: %zu\nbenchmark\n  cycles: %d\n",
                iw, ih, s.st, ow, oh, d.st, cycles);

    // one cycle = Y + U + V, resizers constructed inside (as IQOLanczosResizer::resize, :206-229)
    struct Set {
        iqo::LanczosResizer *ly, *lc;
        iqo::AreaResizer *ay, *ac;
        iqo::LinearResizer *ny, *nc;
    } set = {0, 0, 0, 0, 0, 0};
    auto make = [&]() {
        if (method == "lanczos") {
            set.ly = new iqo::LanczosResizer(degree, iw, ih, ow, oh, 1);
            set.lc = new iqo::LanczosResizer(degree, iw / 2, ih / 2, ow / 2, oh / 2, 2);
        } else if (method == "area") {
            set.ay = new iqo::AreaResizer(iw, ih, ow, oh);
            set.ac = new iqo::AreaResizer(iw / 2, ih / 2, ow / 2, oh / 2);
        } else {
            set.ny = new iqo::LinearResizer(iw, ih, ow, oh);
            set.nc = new iqo::LinearResizer(iw / 2, ih / 2, ow / 2, oh / 2);
        }
    };
    auto drop = [&]() {
        delete set.ly;
        delete set.lc;
        delete set.ay;
        delete set.ac;
        delete set.ny;
        delete set.nc;
        set = Set{0, 0, 0, 0, 0, 0};
    };
    auto run = [&]() {
        const uint8_t *sb = s.buf.data();
        uint8_t *db = d.buf.data();
        if (set.ly) {
            set.ly->resize(s.st, sb + s.y(), d.st, db + d.y());
            set.lc->resize(s.st / 2, sb + s.u(), d.st / 2, db + d.u());
            set.lc->resize(s.st / 2, sb + s.v(), d.st / 2, db + d.v());
        } else if (set.ay) {
            set.ay->resize(s.st, sb + s.y(), d.st, db + d.y());
            set.ac->resize(s.st / 2, sb + s.u(), d.st / 2, db + d.u());
            set.ac->resize(s.st / 2, sb + s.v(), d.st / 2, db + d.v());
        } else {
            set.ny->resize(s.st, sb + s.y(), d.st, db + d.y());
            set.nc->resize(s.st / 2, sb + s.u(), d.st / 2, db + d.u());
            set.nc->resize(s.st / 2, sb + s.v(), d.st / 2, db + d.v());
        }
    };
    double best = 1e30;
    if (reuse)
        make();
    for (int c = 0; c < cycles; ++c) {
        auto t0 = std::chrono::high_resolution_clock::now();
        if (!reuse)
            make();
        run();
        if (!reuse)
            drop();
        auto t1 = std::chrono::high_resolution_clock::now();
        best = std::min(best, std::chrono::duration<double>(t1 - t0).count());
    }
    if (reuse)
        drop();
    std::printf("  elapsed time: %8.3f ms/cycle\n", best * 1000);
    if (a.count("check")) {
        FILE *f = std::fopen(a["check"].c_str(), "wb");
        if (!f)
            return EIO;
        for (long y = 0; y < oh; ++y)
            std::fwrite(d.buf.data() + d.y() + y * d.st, 1, ow, f);
        std::fclose(f);
    }
    int onHip = 0, onCpu = 0;
    iqo_dropin_backend_counts(&onHip, &onCpu);
    std::printf("  backend: hip %d cpu %d\n", onHip, onCpu);
    return 0;
}
