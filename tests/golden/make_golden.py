#!/usr/bin/env python3
"""Generates tests/golden/cornell_box_screenshot_blocks.json from the reference's committed render
/root/reference/screenshots/cornell_box.png (600x600 RGB8, gamma-2 encoded by util::WriteImage,
Util.cpp:39-79; scene data/cornell_box_original.json; spp not recorded).

The fixture is data: per-block means of the 8-bit values over 30x30 blocks of 20x20 pixels, in
image (top-down) order, plus the image shape. Run here (the reference is not on the GPU box)."""
import json
import os
import sys

import numpy as np
from PIL import Image

SRC = "/root/reference/screenshots/cornell_box.png"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cornell_box_screenshot_blocks.json")
BLOCK = 20


def main():
    img = np.asarray(Image.open(SRC).convert("RGB"), dtype=np.float64)
    h, w, _ = img.shape
    assert h % BLOCK == 0 and w % BLOCK == 0, img.shape
    blocks = img.reshape(h // BLOCK, BLOCK, w // BLOCK, BLOCK, 3).mean(axis=(1, 3)) / 255.0
    json.dump({"source": "reference screenshots/cornell_box.png", "scene": "cornell_box_original.json",
               "shape": [h, w], "block": BLOCK, "encoding": "mean of 8-bit gamma-2 values / 255, top-down rows",
               "blocks": np.round(blocks, 5).tolist()}, open(OUT, "w"))
    print("wrote", OUT, blocks.shape)


if __name__ == "__main__":
    sys.exit(main())
