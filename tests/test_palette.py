"""voxels.txt parsing (och::voxel_data, ORT/och_voxel.cpp:195-305)."""
import numpy as np
import pytest


def test_reference_palette(ort):
    v = ort.VoxelData()
    assert v.get_cnt() == 4
    assert v.get_names() == ["Stone", "Grass", "Dark Grass", "Dirt"]
    c = v.get_colours()
    assert c.shape == (24,)
    assert c[0] == 0xFF5D4444        # Stone x_pos 44445D -> r 0x44 g 0x44 b 0x5D a 0xFF
    assert c[6 * 1 + 5] == 0xFF27853F  # Grass z_neg 3F8527


@pytest.mark.parametrize("text,msg", [
    ("", "did not contain"),
    ("A:\n112233\n", "must contain at least one"),
    ("Stone:\n11223G 0 0 0 0 0", "Non-hex"),
    ("Stone:\n112233\n", "ended unexpectedly"),
    ("ABCDEFGHIJKLMNOPQ:\n", "may not exceed"),
])
def test_palette_errors(ort, tmp_path, text, msg):
    p = tmp_path / "v.txt"
    p.write_text(text)
    with pytest.raises(ort.VoxelDataError, match=msg):
        ort.VoxelData(p)


def test_reload_count_mismatch(ort, tmp_path):
    p = tmp_path / "v.txt"
    p.write_text("Rock:" + " 010203" * 6)
    v = ort.VoxelData(p)
    assert v.get_colours()[0] == 0xFF030201
    p.write_text("Rock:" + " 010203" * 6 + "\nMoss:" + " 040506" * 6)
    with pytest.raises(ort.VoxelDataError, match="does not match"):
        v.reload()
