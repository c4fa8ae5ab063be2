// image.cpp -- host-side PNG scanline reconstruction for the glTF texture loader
// (mpt/image.py).  The reference decodes textures with stb_image (Image8Bit::read_image,
// Image.cpp:33-61, called by ThreadFunctions::load_scene_texture, ThreadFunctions.cpp:30-97);
// the loader restates the PNG part of it: zlib inflate in Python's zlib, the per-row filter
// reversal here (sequential along a row: Python would take seconds on a 4K texture).
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "mpt.h"

namespace mpt {
int api_fail(int code, const char* msg);   // mpt_api.cpp: sets mpt_last_error
}

extern "C" int mpt_png_unfilter(const uint8_t* filtered, int64_t filtered_size, uint8_t* out, int32_t rows,
                                int32_t row_bytes, int32_t bpp) {
    if (!filtered || (!out && rows > 0)) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (rows < 0 || row_bytes < 0 || bpp < 1 || bpp > 8)
        return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "png: bad geometry");
    if (filtered_size < (int64_t)rows * (row_bytes + 1)) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "png: truncated image data");
    const uint8_t* prev = nullptr;
    for (int32_t y = 0; y < rows; y++) {
        const uint8_t* src = filtered + (size_t)y * (row_bytes + 1);
        uint8_t* dst = out + (size_t)y * row_bytes;
        const int type = src[0];
        src++;
        switch (type) {
        case 0:   // None
            std::memcpy(dst, src, (size_t)row_bytes);
            break;
        case 1:   // Sub
            for (int32_t i = 0; i < row_bytes; i++) dst[i] = (uint8_t)(src[i] + (i >= bpp ? dst[i - bpp] : 0));
            break;
        case 2:   // Up
            for (int32_t i = 0; i < row_bytes; i++) dst[i] = (uint8_t)(src[i] + (prev ? prev[i] : 0));
            break;
        case 3:   // Average
            for (int32_t i = 0; i < row_bytes; i++) {
                const int a = i >= bpp ? dst[i - bpp] : 0, b = prev ? prev[i] : 0;
                dst[i] = (uint8_t)(src[i] + ((a + b) >> 1));
            }
            break;
        case 4:   // Paeth
            for (int32_t i = 0; i < row_bytes; i++) {
                const int a = i >= bpp ? dst[i - bpp] : 0, b = prev ? prev[i] : 0;
                const int c = (i >= bpp && prev) ? prev[i - bpp] : 0;
                const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                const int pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                dst[i] = (uint8_t)(src[i] + pred);
            }
            break;
        default:
            return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "png: bad filter type");
        }
        prev = dst;
    }
    return MPT_OK;
}
