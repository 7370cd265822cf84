"""PosedImage (the evaluation views, reference data/datasets.py:376-712) against the reference's own
class run on the same directories (tests/golden/posed_*.npz, make_golden.gen_posed): 8- and 16-bit
PNG (every scanline filter type), grey / grey + alpha / RGB / RGBA, 16-bit with a ``bit_depth`` of
10, PIL-written PNG, float32 linear renders, synthetic display / linear and real captures, alpha over
white, Bayer (RGB) and monochrome (grey) sensors, ``camera_angle_x`` and ``intrinsics``, exposure
time and gain, permutations, a ``views/`` folder one level above the dataset.

cv2 is absent from both sides: the reference ran with imread returning the samples each file holds
(in OpenCV's BGR order) and cvtColor restated (make_golden.install_cv2), so these fixtures pin the
reference's PosedImage code and this package's file decoding; OpenCV's own grey conversion is
parity unpinned.  Quantised views must be bit-identical (torch.equal); the float32 linear renders
within 1 ulp (the fixture ran under numpy 2, whose promotion adds the float64 log_eps in float64,
where the reference's numpy 1.24 -- and this package -- add it in float32)."""
import glob
import os
import tempfile

import numpy as np
import pytest
import torch

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(os.path.basename(p)[len("posed_"):-len(".npz")] for p in glob.glob(os.path.join(GOLDEN, "posed_*.npz")))


def build_views_dir(z):
    """Recreate the fixture's dataset directory from its ``file:`` entries -> the dataset root."""
    top = tempfile.mkdtemp(prefix="den_posed_")
    for k in z.files:
        if k.startswith("file:"):
            path = os.path.join(top, k[len("file:"):])
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "wb") as f:
                f.write(z[k].tobytes())
    return os.path.normpath(os.path.join(top, str(z["root"])))


def test_cases_present():
    assert len(CASES) >= 8, CASES


@pytest.mark.parametrize("case", CASES)
def test_posed_image_matches_reference(case):
    from deblur_e_nerf.data.datasets import PosedImage
    z = np.load(os.path.join(GOLDEN, f"posed_{case}.npz"))
    root = build_views_dir(z)
    linear = "linear" in case
    for i in range(int(z["n_runs"])):
        p = f"run{i}:"
        perm = int(z[p + "perm"])
        pi = PosedImage(root, str(z[p + "stage"]), None if perm < 0 else perm, bool(z[p + "alpha"]))
        keys = sorted(k[len(p):] for k in z.files if k.startswith(p) and not k.endswith("_dtype")
                      and k[len(p):] not in ("stage", "perm", "alpha", "min_normalized_pixel_value",
                                             "max_normalized_pixel_value"))
        assert sorted(pi.posed_imgs.keys()) == keys, (sorted(pi.posed_imgs.keys()), keys)
        for k in keys:
            got, ref = pi.posed_imgs[k], torch.from_numpy(z[p + k])
            assert str(got.dtype) == str(z[p + k + "_dtype"]), (case, i, k, got.dtype)
            assert got.shape == ref.shape, (case, i, k, got.shape, ref.shape)
            if k == "img" and linear:
                ulp = torch.finfo(torch.float32).eps * ref.abs().clamp_min(1e-3)
                assert bool(((got - ref).abs() <= ulp).all()), (case, i, float((got - ref).abs().max()))
            else:
                assert torch.equal(got, ref), (case, i, k, float((got.double() - ref.double()).abs().max()))
        lo, hi = float(z[p + "min_normalized_pixel_value"]), float(z[p + "max_normalized_pixel_value"])
        assert pi.min_normalized_pixel_value == lo
        if linear:
            assert abs(pi.max_normalized_pixel_value - hi) <= 2e-7 * hi
        else:
            assert pi.max_normalized_pixel_value == hi
        # the dataset protocol the DataModule's loader uses
        item = pi[0]
        assert set(item) == set(keys) - {"intrinsics"}
        assert len(pi) == z[p + "img"].shape[0]


def test_sample_ids_round_trip():
    """The space-padded 16 code points become the file names again (deblur_e_nerf.py:1310-1319)."""
    from deblur_e_nerf.data.datasets import PosedImage
    from deblur_e_nerf.models.deblur_e_nerf import DeblurENeRF
    z = np.load(os.path.join(GOLDEN, "posed_mono_display_rgba8.npz"))
    pi = PosedImage(build_views_dir(z), "val", None, False)
    names = DeblurENeRF.unicode_code_pt_tensor_to_str(pi.posed_imgs.sample_id)
    assert names[0] == "r_0" and names[1] == "view_long_name1" and len(pi.posed_imgs.sample_id[0]) == 16


def test_png_decoder_all_filters_and_depths():
    """utils/image_io against arrays encoded with every filter type: 16-bit colour through
    den_png_unfilter (host code in libden.so), the rest through PIL; OpenCV's channel conventions."""
    from deblur_e_nerf.utils import image_io
    import sys
    sys.path.insert(0, GOLDEN)
    import pngenc
    g = np.random.default_rng(0)
    d = tempfile.mkdtemp(prefix="den_png_")
    for depth in (8, 16):
        for C in (1, 2, 3, 4):
            a = g.integers(0, 2 ** depth, size=(13, 17, C) if C > 1 else (13, 17)).astype(
                np.uint16 if depth == 16 else np.uint8)
            path = os.path.join(d, f"x{depth}_{C}.png")
            with open(path, "wb") as f:
                f.write(pngenc.encode_png(a, depth))
            got = image_io.imread_unchanged(path)
            exp = pngenc.bgr(a)
            assert got.dtype == exp.dtype and got.shape == exp.shape and np.array_equal(got, exp), (depth, C)


def test_imwrite_round_trip():
    from deblur_e_nerf.utils import image_io
    d = tempfile.mkdtemp(prefix="den_png_")
    g = np.random.default_rng(1)
    for a in (g.integers(0, 256, (9, 11)).astype(np.uint8), g.integers(0, 256, (9, 11, 1)).astype(np.uint8),
              g.integers(0, 256, (9, 11, 3)).astype(np.uint8)):
        p = os.path.join(d, "p.png")
        image_io.imwrite(p, a)
        back = image_io.imread_unchanged(p)
        assert np.array_equal(back, a[..., 0] if a.ndim == 3 and a.shape[2] == 1 else a)


def test_missing_views_and_bad_inputs():
    from deblur_e_nerf.data.datasets import PosedImage
    d = tempfile.mkdtemp(prefix="den_noviews_")
    assert PosedImage.posed_img_folder_path(d) is None
    with pytest.raises(FileNotFoundError):
        PosedImage(d, "val", None)
    # a real capture with an alpha channel is refused, as the reference asserts (datasets.py:604-605)
    z = np.load(os.path.join(GOLDEN, "posed_mono_display_rgba8.npz"))
    root = build_views_dir(z)
    os.remove(os.path.join(root, "renderer_params.npz"))
    with pytest.raises(AssertionError):
        PosedImage(root, "val", None, False)
