// Sanitizer driver for host/image_io.cpp (TEST INFRASTRUCTURE): built with
// -fsanitize=address,undefined by tests/test_sanitizers.py, it reads every
// file named on the command line through the public EXR entry points.  A
// malformed file must come back as an error status, never as an
// out-of-bounds access, overflow or crash (which the sanitizers abort on).
#include <cstdio>
#include <vector>

#include "image_io.h"

int main(int argc, char** argv) {
    int rejected = 0;
    for (int i = 1; i < argc; ++i) {
        int w = 0, h = 0, ch = 0;
        if (bmfr_exr_info(argv[i], &w, &h, &ch) != 0) {
            ++rejected;
            continue;
        }
        if (w <= 0 || h <= 0 || (long long)w * h > (1LL << 24)) {  // keep the buffer bounded
            ++rejected;
            continue;
        }
        std::vector<float> rgb((size_t)w * h * 3);
        if (bmfr_exr_read_rgb(argv[i], w, h, rgb.data()) != 0) ++rejected;
    }
    std::printf("files %d rejected %d\n", argc - 1, rejected);
    return 0;
}
