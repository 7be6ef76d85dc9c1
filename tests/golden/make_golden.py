#!/usr/bin/env python3
"""Generates the screenshot fixtures from the reference's committed renders (600x600 RGB8, gamma-2
encoded by util::WriteImage, Util.cpp:39-79; spp not recorded):
  tests/golden/cornell_box_screenshot_blocks.json   <- screenshots/cornell_box.png
      (scene data/cornell_box_original.json)
  tests/golden/final_scene2_screenshot_blocks.json  <- screenshots/final_scene2.png
      (scene data/book2_final_scene_10000_samples.json; its ground heights and cube sphere centres
       are random draws that need not match the shipped JSON)

A fixture is data: per-block means of the 8-bit values over 30x30 blocks of 20x20 pixels, in image
(top-down) order, plus the image shape. Run here (the reference is not on the GPU box)."""
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
SHOTS = [("cornell_box.png", "cornell_box_original.json", "cornell_box_screenshot_blocks.json"),
         ("final_scene2.png", "book2_final_scene_10000_samples.json", "final_scene2_screenshot_blocks.json")]
BLOCK = 20


def main():
    for png, scene, out in SHOTS:
        img = np.asarray(Image.open("/root/reference/screenshots/" + png).convert("RGB"), dtype=np.float64)
        h, w, _ = img.shape
        assert h % BLOCK == 0 and w % BLOCK == 0, img.shape
        blocks = img.reshape(h // BLOCK, BLOCK, w // BLOCK, BLOCK, 3).mean(axis=(1, 3)) / 255.0
        json.dump({"source": "reference screenshots/" + png, "scene": scene, "shape": [h, w], "block": BLOCK,
                   "encoding": "mean of 8-bit gamma-2 values / 255, top-down rows",
                   "blocks": np.round(blocks, 5).tolist()}, open(os.path.join(HERE, out), "w"))
        print("wrote", out, blocks.shape)


if __name__ == "__main__":
    sys.exit(main())
