// iqo_resize_yuv420p -- file tool: resize raw I420 (YUV 4:2:0 planar) frames on the MI355X
// backend.  Same command line and file layout as the reference's sample tool
// (sample/resize_yuv420p.cpp:36-191):
//
//   iqo_resize_yuv420p -m method -i in.yuv -iw W -ih H -o out.yuv -ow w -oh h [-frames N]
//   method: linear | area | lanczos[1-9]   (plain "lanczos" = degree 2, as the reference)
//
// File layout (reference :67-76): the luma plane has stride W + W%2 and H + H%2 rows; U and V
// follow, each (stride/2) x (rows/2).  Chroma planes are resized as (stride/2) x (rows/2) images
// (reference :128-160), Lanczos chroma with pxScale 2.
//
// Differences from the reference (extensions only; one frame behaves identically):
//   * -frames N processes N consecutive frames of the file (default 1).
//   * When every plane size is exactly half the luma size (even W, H, w, h) the three planes go
//     through one YUV420 plan (iqo_hip_plan_yuv420, one pipelined call per frame); otherwise the
//     three drop-in resizer objects are used, as in the reference.
//   * Errors return a nonzero exit status with a message (the reference returns errno).
#include <iqo_hip.h>
#include <libiqo/iqo.hpp>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace {

struct I420 {
    size_t w, h;          // picture size
    size_t stX, stY;      // padded luma stride / row count (even)
    size_t sizeY() const { return stX * stY; }
    size_t sizeC() const { return sizeY() / 4; }
    size_t bytes() const { return sizeY() + 2 * sizeC(); }
    static I420 of(size_t w, size_t h) { return I420{w, h, w + w % 2, h + h % 2}; }
};

bool flag(std::map<std::string, std::string> &a, const char *k, std::string &v)
{
    auto it = a.find(k);
    if (it == a.end())
        return false;
    v = it->second;
    return true;
}

int usage()
{
    std::printf("usage: iqo_resize_yuv420p -m method -i input.yuv -iw in_width -ih in_height "
                "-o output.yuv -ow out_width -oh out_height [-frames N]\n"
                "method: linear, area or lanczos[1-9]\n");
    return EINVAL;
}

} // namespace

int main(int argc, char **argv)
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
    std::string method, inPath, outPath, s;
    flag(a, "m", method);
    flag(a, "i", inPath);
    flag(a, "o", outPath);
    long iw = flag(a, "iw", s) ? std::atol(s.c_str()) : 0;
    long ih = flag(a, "ih", s) ? std::atol(s.c_str()) : 0;
    long ow = flag(a, "ow", s) ? std::atol(s.c_str()) : 0;
    long oh = flag(a, "oh", s) ? std::atol(s.c_str()) : 0;
    long frames = flag(a, "frames", s) ? std::atol(s.c_str()) : 1;
    if (inPath.empty() || outPath.empty() || iw <= 0 || ih <= 0 || ow <= 0 || oh <= 0 || frames < 1)
        return usage();

    unsigned degree = 2;
    int m;
    if (method.compare(0, 7, "lanczos") == 0 && method.size() <= 8) {
        if (method.size() == 8) {
            int dg = method[7] - '0';
            if (dg < 1 || dg > 9) {
                std::printf("invalid method: %s\n", method.c_str());
                return EINVAL;
            }
            degree = static_cast<unsigned>(dg);
        }
        m = IQO_METHOD_LANCZOS;
    } else if (method == "area") {
        m = IQO_METHOD_AREA;
    } else if (method == "linear") {
        m = IQO_METHOD_LINEAR;
    } else {
        std::printf("invalid method: %s\n", method.c_str());
        return EINVAL;
    }

    const I420 si = I420::of(iw, ih), di = I420::of(ow, oh);
    std::printf("method: %s\n", m == IQO_METHOD_LANCZOS ? "lanczos" : method.c_str());
    if (m == IQO_METHOD_LANCZOS)
        std::printf("quality\n  degree: %u\n", degree);
    std::printf("backend\n  %s\n", iqo_hip_version());
    std::printf("input\n    path: %s\n    size: %ldx%ld\n  stride: %zux%zu\n", inPath.c_str(), iw, ih, si.stX, si.stY);
    std::printf("output\n    path: %s\n    size: %ldx%ld\n  stride: %zux%zu\n", outPath.c_str(), ow, oh, di.stX,
                di.stY);

    std::FILE *in = std::fopen(inPath.c_str(), "rb");
    if (!in) {
        int e = errno;
        std::perror("fopen");
        std::printf("Could not open \"%s\".\n", inPath.c_str());
        return e ? e : EIO;
    }
    std::FILE *out = std::fopen(outPath.c_str(), "wb");
    if (!out) {
        int e = errno;
        std::perror("fopen");
        std::printf("Could not open \"%s\".\n", outPath.c_str());
        std::fclose(in);
        return e ? e : EIO;
    }

    // Even everywhere -> the chroma planes are exactly W/2 x H/2: one YUV420 plan does all three.
    const bool fused = iw % 2 == 0 && ih % 2 == 0 && ow % 2 == 0 && oh % 2 == 0;
    iqo_hip_yuv_plan *yuv = nullptr;
    if (fused) {
        int st = iqo_hip_plan_yuv420(m, degree, iw, ih, ow, oh, 0, &yuv);
        if (st != IQO_HIP_OK) {
            std::printf("iqo_hip_plan_yuv420: %s\n", iqo_hip_strerror(st));
            std::fclose(in);
            std::fclose(out);
            return EIO;
        }
    }
    // Otherwise the reference's composition: luma resizer + one chroma resizer used twice.
    const size_t scw = si.stX / 2, sch = si.stY / 2, dcw = di.stX / 2, dch = di.stY / 2;
    std::unique_ptr<iqo::LanczosResizer> lY, lC;
    std::unique_ptr<iqo::AreaResizer> aY, aC;
    std::unique_ptr<iqo::LinearResizer> nY, nC;
    if (!fused) {
        if (m == IQO_METHOD_LANCZOS) {
            lY.reset(new iqo::LanczosResizer(degree, iw, ih, ow, oh));
            lC.reset(new iqo::LanczosResizer(degree, scw, sch, dcw, dch, 2));
        } else if (m == IQO_METHOD_AREA) {
            aY.reset(new iqo::AreaResizer(iw, ih, ow, oh));
            aC.reset(new iqo::AreaResizer(scw, sch, dcw, dch));
        } else {
            nY.reset(new iqo::LinearResizer(iw, ih, ow, oh));
            nC.reset(new iqo::LinearResizer(scw, sch, dcw, dch));
        }
    }
    auto plane = [&](bool luma, size_t sst, const uint8_t *sp, size_t dst, uint8_t *dp) {
        if (lY)
            (luma ? lY : lC)->resize(sst, sp, dst, dp);
        else if (aY)
            (luma ? aY : aC)->resize(sst, sp, dst, dp);
        else
            (luma ? nY : nC)->resize(sst, sp, dst, dp);
    };

    std::vector<uint8_t> src(si.bytes()), dst(di.bytes(), 0);
    int rc = 0;
    for (long f = 0; f < frames && rc == 0; ++f) {
        size_t got = std::fread(src.data(), 1, src.size(), in);
        if (got < src.size()) {
            std::perror("fread");
            std::printf("Could not read %zu bytes (frame %ld).\n", src.size(), f);
            rc = EIO;
            break;
        }
        const uint8_t *sY = src.data(), *sU = sY + si.sizeY(), *sV = sU + si.sizeC();
        uint8_t *dY = dst.data(), *dU = dY + di.sizeY(), *dV = dU + di.sizeC();
        if (fused) {
            int st = iqo_hip_resize_yuv420(yuv, si.stX, sY, scw, sU, sV, di.stX, dY, dcw, dU, dV);
            if (st != IQO_HIP_OK) {
                std::printf("iqo_hip_resize_yuv420: %s\n", iqo_hip_strerror(st));
                rc = EIO;
                break;
            }
        } else {
            plane(true, si.stX, sY, di.stX, dY);
            plane(false, scw, sU, dcw, dU);
            plane(false, scw, sV, dcw, dV);
        }
        if (std::fwrite(dst.data(), 1, dst.size(), out) < dst.size()) {
            std::perror("fwrite");
            std::printf("Could not write %zu bytes.\n", dst.size());
            rc = EIO;
        }
    }
    const bool usedYuv = yuv != nullptr;
    if (yuv)
        iqo_hip_yuv_plan_destroy(yuv);
    int onHip = 0, onCpu = 0;
    iqo_dropin_backend_counts(&onHip, &onCpu);
    std::printf("backend: hip %d cpu %d (YUV420 plan: %s)\n", onHip, onCpu, usedYuv ? "yes" : "no");
    std::fclose(in);
    if (std::fclose(out) != 0 && rc == 0)
        rc = EIO;
    return rc;
}
