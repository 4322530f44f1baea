// oracle/ref/ref_ppm.cpp — TEST INFRASTRUCTURE ONLY.
// Writes a W x H float32 RGB framebuffer (row-major, row 0 = top) through the reference
// ppm_p6 writer (HW1/ppm_p6_lib/src/ppm_p6.cpp:257-301) with its default WriteOptions
// (maxval 255, clamp, gamma2 = sqrt, no flip; ppm_p6.hpp:46-51), or with an explicit
// maxval/gamma, so tests/golden holds the reference's own P6 bytes.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "ppm_p6.hpp"

int main(int argc, char** argv) {
    if (argc < 5) { std::fprintf(stderr, "usage: ref_ppm in.f32 W H out.ppm [maxval gamma2]\n"); return 2; }
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    std::vector<float> fb((size_t)W * H * 3);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(fb.data(), sizeof(float), fb.size(), f) != fb.size()) return 1;
    std::fclose(f);
    ppm_p6::Image img(W, H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float* p = &fb[((size_t)y * W + x) * 3];
            ppm_p6::Color c;
            c.r = p[0]; c.g = p[1]; c.b = p[2];
            img.set(x, y, c);
        }
    ppm_p6::WriteOptions opt;
    if (argc > 5) opt.maxval = std::atoi(argv[5]);
    if (argc > 6) opt.gamma2 = std::atoi(argv[6]) != 0;
    std::string err;
    if (!ppm_p6::write_p6(argv[4], img, opt, &err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
    return 0;
}
