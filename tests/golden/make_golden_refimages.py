"""Grey fixtures from the reference's own test images (run in the build container, where /root/reference exists;
the GPU box reads only the committed .npz).

  tests/test_data/images/image_1.png       1920 x 1080 RGB (a real street texture)
  tests/test_data/camera/undistort_input.png  1280 x 960 RGB (tests/test_camera.cpp:115 reads it)

Converted with OpenCV's cv::COLOR_RGB2GRAY fixed-point rule for 8-bit images, Y = (4899 R + 9617 G + 1868 B +
2^13) >> 14 (the 0.299 / 0.587 / 0.114 weights scaled by 2^14).  The grey bytes are an INPUT fixture: the parity
bar of the tests that use them is the GPU path against the oracle on these same bytes; whether OpenCV's imread
(IMREAD_GRAYSCALE goes through libpng's own rgb_to_gray) would give the same bytes is not claimed (parity of the
conversion itself unpinned; it is not on the hot path).

usage: python3 tests/golden/make_golden_refimages.py [reference root]
"""
import os
import sys

import numpy as np
from PIL import Image

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refimages.npz")


def grey(path):
    rgb = np.asarray(Image.open(path).convert("RGB"), dtype=np.uint32)
    y = (4899 * rgb[..., 0] + 9617 * rgb[..., 1] + 1868 * rgb[..., 2] + (1 << 13)) >> 14
    return np.ascontiguousarray(y.astype(np.uint8))


if __name__ == "__main__":
    imgs = {"image_1": grey(os.path.join(REF, "tests/test_data/images/image_1.png")),
            "undistort_input": grey(os.path.join(REF, "tests/test_data/camera/undistort_input.png"))}
    np.savez_compressed(OUT, **imgs)
    for k, v in imgs.items():
        print(k, v.shape, v.dtype, int(v.min()), int(v.max()))
    print("wrote", OUT, os.path.getsize(OUT), "bytes")
