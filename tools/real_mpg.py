"""Reference-encoded .mpg files at benchmark sizes (this container only: needs oracle/_ref/mjref_app,
`make -C oracle ref`).  The reference's own encoder (mjpeg423_encode) codes synthetic camera frames
(oracle/gen_golden.py:synth_rgb scenes), so the P-frames carry the coefficient statistics the
reference writes -- mostly DC-only or empty blocks -- unlike tools/mpg_synth.py's random ones.

  python tools/real_mpg.py static 1920 1080 24 24 realdata/static_1080p.mpg
  python tools/real_mpg.py pan    1920 1080 24 24 realdata/pan_1080p.mpg

static: a fixed scene, a slow brightness drift, moving objects and fresh sensor noise per frame;
pan: the scene moving 3 pixels a frame, plus the same objects and noise; clean: static without the
noise (rendered or denoised content).  Output only; the files stay
out of git (realdata/ is ignored) and travel to the GPU box with the tree."""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
from gen_golden import REF_APP, synth_rgb, write_bmp24  # noqa: E402


def frames(kind, w, h, n, seed=7):
    rng = np.random.default_rng(seed)
    for f in range(n):
        shift = 3 * f if kind == "pan" else 0
        base = synth_rgb(np.random.default_rng(seed), w, h, shift=shift)  # the same scene every frame
        rgb = np.stack([(base >> 16) & 255, (base >> 8) & 255, base & 255], -1).astype(np.int32)
        rgb += f % 5 if kind in ("static", "clean") else 0
        for j in range(3):  # moving objects
            s = 24 + 16 * j
            x0 = (7 * f + 300 * j) % (w - s)
            y0 = (3 * f + 200 * j) % (h - s)
            rgb[y0:y0 + s, x0:x0 + s] = [250 - 5 * (f % 40), 40 + 3 * j, 90 + 50 * j]
        if kind != "clean":
            rgb = rgb + rng.normal(0, 2.0, size=rgb.shape)  # sensor noise, fresh per frame
        yield np.clip(rgb, 0, 255).astype(np.uint8)


def main():
    kind, w, h, n, max_i, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    if not os.path.exists(REF_APP):
        sys.exit(f"{REF_APP} missing: run `make -C oracle ref` first (needs /root/reference)")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        for f, rgb in enumerate(frames(kind, w, h, n)):
            write_bmp24(os.path.join(td, f"in{f:04d}.bmp"), rgb)
        subprocess.run([REF_APP, "encode", str(n), "0", "1", str(max_i), str(w), str(h),
                        os.path.join(td, "in0000.bmp"), out], check=True, capture_output=True)
    print(out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
