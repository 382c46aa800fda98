"""Where the whole-file decoder's time goes (measurements only, GPU box): one seeded synthetic
.mpg (tools/mpg_synth), then in one process
  - library load, context creation (HIP init + code-object load),
  - per chunk size: pipeline create / decode with a no-op sink / decode with the BMP sink /
    destroy, with the pipeline's own stats (front-end busy, sink busy, GPU span),
  - mj423_decode_file (mjpeg423_decode) warm, i.e. after the first call paid HIP init.
One JSON line per measurement on stdout.

  python tools/file_decode_probe.py W H FRAMES [CHUNK ...]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mjpeg423-video-decoder-software_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import mpg_synth  # noqa: E402

import mj423  # noqa: E402


def main():
    w, h, n = (int(x) for x in sys.argv[1:4])
    chunks = [int(x) for x in sys.argv[4:]] or [0]
    work = f"/tmp/mj423_probe_{os.getpid()}"
    os.makedirs(work, exist_ok=True)
    src = os.path.join(work, "in.mpg")
    mpg_synth.build()
    mpg_synth.write(src, w, h, n, gop=24)
    t = time.perf_counter()
    mj423.lib()
    t_lib = time.perf_counter() - t
    t = time.perf_counter()
    ctx = mj423.Context()
    t_ctx = time.perf_counter() - t
    print(json.dumps({"what": "init", "lib_load_s": round(t_lib, 4), "ctx_create_s": round(t_ctx, 4)}), flush=True)
    m = mj423.Mpg(src)
    for chunk in chunks:
        t = time.perf_counter()
        p = mj423.Pipeline(ctx, w, h, chunk_frames=chunk)
        t_create = time.perf_counter() - t
        res = {"what": "pipeline", "geometry": f"{w}x{h}", "frames": n, "chunk_arg": chunk,
               "create_s": round(t_create, 4)}
        for label, sink in (("noop", lambda fi, v: 0),
                            ("bmp", lambda fi, v: mj423.write_bmp(os.path.join(work, f"o{fi:04d}.bmp"), v))):
            for rep in range(2):
                t = time.perf_counter()
                st = p.decode(m, 0, n, sink)
                wall = time.perf_counter() - t
                res[f"{label}{rep}"] = {"wall_s": round(wall, 4), "chunks": st.chunks,
                                        "frontend_busy_s": round(st.frontend_busy_s, 4),
                                        "sink_busy_s": round(st.sink_busy_s, 4),
                                        "gpu_span_ms": round(st.gpu_span_ms, 3)}
        t = time.perf_counter()
        p.close()
        res["destroy_s"] = round(time.perf_counter() - t, 4)
        print(json.dumps(res), flush=True)
    m.close()
    for rep in range(2):
        t = time.perf_counter()
        mj423.decode_file(src, os.path.join(work, "d0000.bmp"))
        print(json.dumps({"what": "decode_file", "rep": rep, "wall_s": round(time.perf_counter() - t, 4)}), flush=True)
    for f in os.listdir(work):
        os.remove(os.path.join(work, f))
    os.rmdir(work)


if __name__ == "__main__":
    main()
