/*
 * ref_app.c -- TEST INFRASTRUCTURE ONLY.  A command-line wrapper (ours) around the
 * reference's own top-level codec functions, compiled in place from /root/reference
 * by `make -C oracle ref` into oracle/_ref/mjref_app:
 *   mjref_app encode <num_frames> <first> <stride> <max_I_interval> <w> <h> <in_base####.bmp> <out.mpg>
 *       -> mjpeg423_encode()  (mj/encoder/mjpeg423_encoder.c:18)
 *   mjref_app decode <in.mpg> <out_base####.bmp>
 *       -> mjpeg423_decode()  (mj/decoder/mjpeg423_decoder.c:20)
 * Used by oracle/gen_golden.py to make the .mpg stream and BMP golden files.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "decoder/mjpeg423_decoder.h"
#include "encoder/mjpeg423_encoder.h"

int main(int argc, char **argv)
{
    if (argc == 10 && strcmp(argv[1], "encode") == 0) {
        mjpeg423_encode((uint32_t)atoi(argv[2]), atoi(argv[3]), atof(argv[4]), (uint32_t)atoi(argv[5]),
                        (uint32_t)atoi(argv[6]), (uint32_t)atoi(argv[7]), argv[8], argv[9]);
        return 0;
    }
    if (argc == 4 && strcmp(argv[1], "decode") == 0) {
        mjpeg423_decode(argv[2], argv[3]);
        return 0;
    }
    fprintf(stderr, "usage: %s encode n first stride maxI w h in####.bmp out.mpg | decode in.mpg out####.bmp\n", argv[0]);
    return 2;
}
