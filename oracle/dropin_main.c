/*
 * dropin_main.c -- TEST INFRASTRUCTURE: the drop-in builds of INTEGRATION.md, made by
 * `make -C oracle dropin` into oracle/_ref/ and run by tests/test_gpu_parity.py:
 *
 *   mjdrop_blocks: the reference's own decoder (mj/decoder/mjpeg423_decoder.c,
 *                  lossless_decode.c, libbmp) compiled in place, with ITS idct.c and
 *                  ycbcr_to_rgb.c left out -- idct()/ycbcr_to_rgb() come from
 *                  libmj423gpu.so (zero source changes);
 *   mjdrop_file:   this file alone against libmj423gpu.so, whose mjpeg423_decode() is the
 *                  whole GPU decoder.
 *
 *   usage: mjdrop_* <in.mpg> <out_base0000.bmp>
 */
#include <stdio.h>

/* mj/decoder/mjpeg423_decoder.h:14 (and include/mj423io.h) */
void mjpeg423_decode(const char *filename_in, const char *filenamebase_out);

int main(int argc, char **argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s in.mpg out0000.bmp\n", argv[0]);
        return 2;
    }
    mjpeg423_decode(argv[1], argv[2]);
    return 0;
}
