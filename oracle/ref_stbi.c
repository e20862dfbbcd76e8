/* Test infrastructure: the reference's own image decoder, stb_image as the
 * reference vendors it (src/lib/image_utils/stb_image.h, used by
 * image_utils.cpp:4-5, 22-23), compiled from where it lies under
 * /root/reference by oracle/Makefile into oracle/_ref/ (never copied, never
 * shipped). tests/test_assets_stb.py compares the package's PIL decode of
 * the reference's assets with it. */
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"

/* stbi_load(path, &w, &h, &ch, 0) after stbi_set_flip_vertically_on_load(flip)
 * (image_utils.cpp:22-23); the caller frees with ref_stbi_free. */
unsigned char* ref_stbi_load(const char* path, int flip, int* w, int* h, int* ch) {
    stbi_set_flip_vertically_on_load(flip);
    return stbi_load(path, w, h, ch, 0);
}

void ref_stbi_free(unsigned char* p) { stbi_image_free(p); }
