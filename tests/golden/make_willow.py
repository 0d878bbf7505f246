"""Convert the reference's willow map (maps/willow-full-0.05.pgm + .yaml) into
a compact occupancy fixture, tests/golden/willow_walls.npz.

The GPU box has no /root/reference, so config 4 reads this
fixture instead. map_server semantics (negate: 0): occupancy = (255 - p)/255,
occupied above occupied_thresh = 0.5. Row 0 of a PGM is the top of the map:
the mask is flipped so that row index = map y. Data only: the mask, the shape,
the resolution and the yaml origin.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "roborts-edu-slam_amd"))

from roborts_csm.worlds import read_pgm  # noqa: E402

SRC = "/root/reference/maps/willow-full-0.05.pgm"


def main():
    p = read_pgm(SRC)
    occ = (255.0 - p.astype(np.float64)) / 255.0
    wall = np.ascontiguousarray((occ > 0.5)[::-1])
    np.savez_compressed(os.path.join(HERE, "willow_walls.npz"), wall_bits=np.packbits(wall),
                        shape=np.array(wall.shape), resolution=0.05,
                        origin=np.array([-15.025, -28.625, 0.0]))
    print("willow", wall.shape, int(wall.sum()), "occupied cells")


if __name__ == "__main__":
    main()
