"""Generate tests/golden/bitshuffle_kiyo.npz with the kiyo-masui bitshuffle
(imagecodecs 2021.8.26 / bitshuffle 0.3.5) shipped in this image's conda
python.  c-blosc2 v2.21.3, which TileDB calls for BITSHUFFLE
(bitshuffle_filter.cc:146-149) but does not vendor, embeds the same
bitshuffle algorithm; imagecodecs with blocksize=0 processes 8192-byte blocks,
which is TileDB's BSHUF_TARGET_BLOCK_SIZE_B (bitshuffle_filter.cc:48).

Run with: /opt/conda/bin/python3.9 tests/golden/make_bitshuffle_fixtures.py
"""
import os

import numpy as np
import imagecodecs

HERE = os.path.dirname(os.path.abspath(__file__))
rng = np.random.default_rng(20261015)
out = {}
for ts in (1, 2, 4, 8):
    # sizes: multiples of 8*ts (whole groups), partial groups, multi-block
    for nbytes in (8 * ts, 16 * ts, 24 * ts, 8192, 8192 + 64 * ts, 2 * 8192 + 8 * ts * 7):
        data = rng.integers(0, 256, nbytes, dtype=np.uint8)
        enc = imagecodecs.bitshuffle_encode(data.tobytes(), itemsize=ts, blocksize=0)
        out[f"in_ts{ts}_n{nbytes}"] = data
        out[f"out_ts{ts}_n{nbytes}"] = np.frombuffer(enc, dtype=np.uint8)
np.savez_compressed(os.path.join(HERE, "bitshuffle_kiyo.npz"), **out)
print("wrote", len(out) // 2, "vectors;", imagecodecs.__version__)
