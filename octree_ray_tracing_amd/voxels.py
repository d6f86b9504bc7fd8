"""Voxel palette: the reference's voxels.txt format (och::voxel_data).

Mirrors ORT/och_voxel.h:8-27 (format), ORT/och_voxel.cpp:26-60 (get_voxel_cnt:
one voxel per ':'), :195-305 (constructor / reload: name up to ':', then six
RRGGBB colours x_pos..z_neg, alpha 0xFF) with the same error messages.  The
palette is packed as olc::Pixel RGBA8 words (r in the low byte) so it can be
uploaded with GpuPool.set_palette and indexed as colours[6 * (voxel - 1) + dir]
(ORT/test_och_h_octree.cpp:84).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

DEFAULT_VOXELS = Path(__file__).resolve().parent / "data" / "voxels.txt"
NAME_MAX_LEN = 15          # och::name::max_len, ORT/och_voxel.h:38-43


class VoxelDataError(ValueError):
    pass


def _parse(text: str, filename: str):
    count = text.count(":")
    if count == 0:
        raise VoxelDataError("File did not contain a valid voxel")
    pos = 0
    names, colours = [], np.zeros((count, 6), np.uint32)

    def getc():
        nonlocal pos
        if pos >= len(text):
            return None
        c = text[pos]
        pos += 1
        return c

    def first_non_space():
        while True:
            c = getc()
            if c is None or not c.isspace():
                return c

    for vx in range(count):
        c = first_non_space()
        name = []
        i = 0
        while i != NAME_MAX_LEN and c != ":":
            if c is None:
                raise VoxelDataError(f"{filename} ended unexpectedly")
            name.append(c)
            i += 1
            c = getc()
        if i == 1:
            raise VoxelDataError("Voxel-names must contain at least one character")
        if i == NAME_MAX_LEN:
            raise VoxelDataError(f"Voxel-names may not exceed {NAME_MAX_LEN} characters")
        if any(ord(ch) < 32 or ord(ch) == 127 for ch in name):
            raise VoxelDataError(f"Voxel-names may not contain control-characters (see voxel number{vx + 1})")
        names.append("".join(name))
        for d in range(6):
            c = first_non_space()
            rgb = []
            for _ in range(3):
                hexpair = ""
                for _ in range(2):
                    if c is None:
                        raise VoxelDataError(f"{filename} ended unexpectedly")
                    if c not in "0123456789abcdefABCDEF":
                        raise VoxelDataError(f"Non-hex character in colour-value ({names[-1]} at colour no. {d + 1})")
                    hexpair += c
                    c = getc()
                rgb.append(int(hexpair, 16))
            colours[vx, d] = rgb[0] | (rgb[1] << 8) | (rgb[2] << 16) | (0xFF << 24)
            if c is not None:
                pos -= 1            # the reference re-reads from first_non_space
    return names, colours


class VoxelData:
    """och::voxel_data: names and 6 face colours per voxel id (1-based)."""

    def __init__(self, filename: str | Path = DEFAULT_VOXELS):
        self.filename = str(filename)
        self.names, self.colours = _parse(Path(self.filename).read_text(), self.filename)

    def get_cnt(self) -> int:
        return len(self.names)

    def get_names(self) -> list[str]:
        return list(self.names)

    def get_colours(self) -> np.ndarray:
        """(n_voxels * 6,) uint32 RGBA8, x_pos..z_neg per voxel."""
        return self.colours.reshape(-1).copy()

    def reload(self):
        names, colours = _parse(Path(self.filename).read_text(), self.filename)
        if len(names) != len(self.names):
            raise VoxelDataError("New Voxel-count does not match old")
        self.names, self.colours = names, colours
