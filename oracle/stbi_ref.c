/* TEST INFRASTRUCTURE (oracle/_ref): the reference's own image decoder, stb_image.h as the
 * reference ships it (thirdparties/stbi/stb_image.h, unmodified, compiled from where it lies in
 * /root/reference by oracle/Makefile's `ref` target, x86-64 defaults: the SSE2 kernels), behind a
 * small command-line driver.  It generates the golden decodes of tests/golden/images/
 * (tests/golden/make_image_fixtures.py); nothing in the product or on the GPU box runs it.
 *
 * usage: stbi_decode <u8|f32> <req_comp> <flip_y> <in> <out>
 *   u8:  stbi_load   (Image8Bit::read_image, Image.cpp:33-61)
 *   f32: stbi_loadf  (Image32Bit::read_image_hdr, Image.cpp:342-370)
 * out = int32 w, h, comp (the file's channels), then w*h*n values (n = req_comp or comp). */
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv) {
    if (argc != 6) { fprintf(stderr, "usage: %s u8|f32 req_comp flip_y in out\n", argv[0]); return 2; }
    const int req = atoi(argv[2]);
    stbi_set_flip_vertically_on_load(atoi(argv[3]));
    int w = 0, h = 0, comp = 0;
    void* px;
    size_t elem;
    if (strcmp(argv[1], "f32") == 0) { px = stbi_loadf(argv[4], &w, &h, &comp, req); elem = sizeof(float); }
    else { px = stbi_load(argv[4], &w, &h, &comp, req); elem = 1; }
    if (!px) { fprintf(stderr, "stb_image: %s\n", stbi_failure_reason()); return 1; }
    FILE* f = fopen(argv[5], "wb");
    if (!f) return 1;
    const int hdr[3] = {w, h, comp};
    fwrite(hdr, sizeof(int), 3, f);
    fwrite(px, elem, (size_t)w * h * (req ? req : comp), f);
    fclose(f);
    stbi_image_free(px);
    return 0;
}
