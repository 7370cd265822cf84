"""Image files of the evaluation views and of the saved predictions, without OpenCV (absent here).

The reference reads every view with ``cv2.imread(path, cv2.IMREAD_UNCHANGED)`` (data/datasets.py:
504-509) and writes predictions with ``cv2.imwrite`` (models/deblur_e_nerf.py:1047-1053).
``imread_unchanged`` returns what that call returns -- the file's own sample type (uint8, uint16,
float32) and OpenCV's channel conventions:

* grey -> (H, W); grey + alpha -> (H, W, 4) BGRA with B = G = R = grey (OpenCV expands grey + alpha
  to colour); RGB / palette -> (H, W, 3) BGR (a palette's transparency is dropped, as OpenCV's
  three-channel palette decode does); RGBA -> (H, W, 4) BGRA;
* PNG at 1-8 bits (any colour type, interlaced or not) and 16-bit grey PNG are decoded by PIL
  (lossless: the stored integers); 16-bit grey + alpha / RGB / RGBA PNG, which PIL truncates to 8
  bits, by the PNG reader below: zlib inflate, then the scanline unfiltering in libden.so
  (``den_png_unfilter``, host code) and the big-endian samples;
* ``.npy`` float32 arrays (H, W[, 3 | 4], BGR[A] order) stand in for OpenCV's float formats (the
  linear-colour renders of ``renderer_params.npz`` ``interm_color_space = "linear"``); OpenEXR
  files need OpenCV's codec and raise ``DenError``.

``bgr_to_gray`` restates ``cv2.cvtColor(img, cv2.COLOR_BGR2GRAY)`` on float32 images (the reference
casts to float32 first, datasets.py:627-644): OpenCV 4.5.2 (environment.yml:22) computes
fma(r, 0.299f, fma(g, 0.587f, b * 0.114f)) per pixel in its SIMD path; evaluated here in float64
and rounded once, which is that value exactly for 8- and 16-bit inputs (every product and partial
sum is exact in float64).  Parity with OpenCV itself is unpinned (no OpenCV output exists here).
"""
import os
import struct
import zlib

import numpy as np

PNG_SIGNATURE = b"\x89PNG\r\n\x1a\n"
GRAY_COEFFS_BGR = (np.float32(0.114), np.float32(0.587), np.float32(0.299))  # B2YF, G2YF, R2YF


class ImageFormatError(ValueError):
    pass


def _png_header(path):
    """(width, height, bit depth, colour type, interlace) of a PNG file, or None for other files."""
    with open(path, "rb") as f:
        head = f.read(33)
    if head[:8] != PNG_SIGNATURE or head[12:16] != b"IHDR":
        return None
    w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", head[16:29])
    return w, h, depth, ctype, interlace


def _read_png16_color(path, w, h, ctype, interlace):
    """16-bit grey + alpha (4) / RGB (2) / RGBA (6) PNG -> (H, W, 4 | 3 | 4) uint16 in OpenCV's order."""
    from .. import _native
    if interlace:
        raise ImageFormatError(f"{path}: interlaced 16-bit colour PNG is not supported")
    channels = {2: 3, 4: 2, 6: 4}[ctype]
    with open(path, "rb") as f:
        data = f.read()
    pos, idat = 8, []
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        kind = data[pos + 4:pos + 8]
        if kind == b"IDAT":
            idat.append(data[pos + 8:pos + 8 + n])
        elif kind == b"IEND":
            break
        pos += 12 + n
    raw = zlib.decompress(b"".join(idat))
    bpp = 2 * channels
    row_bytes = w * bpp
    if len(raw) != h * (row_bytes + 1):
        raise ImageFormatError(f"{path}: {len(raw)} inflated bytes, expected {h * (row_bytes + 1)}")
    samples = _native.png_unfilter(np.frombuffer(raw, dtype=np.uint8), h, row_bytes, bpp)
    img = samples.view(">u2").astype(np.uint16).reshape(h, w, channels)
    if channels == 2:   # grey + alpha -> BGRA with the grey replicated
        g, a = img[..., 0], img[..., 1]
        return np.stack([g, g, g, a], axis=-1)
    if channels == 3:
        return np.ascontiguousarray(img[..., ::-1])
    return np.ascontiguousarray(img[..., [2, 1, 0, 3]])


def imread_unchanged(path):
    """``cv2.imread(path, cv2.IMREAD_UNCHANGED)`` for the formats above."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npy":
        img = np.load(path, allow_pickle=False)
        if img.ndim not in (2, 3) or (img.ndim == 3 and img.shape[2] not in (3, 4)):
            raise ImageFormatError(f"{path}: expected (H, W[, 3 | 4]), got {img.shape}")
        return img
    if ext == ".exr":
        from .._native import DenError
        raise DenError(f"{path}: OpenEXR views need OpenCV's codec, which this build does not have; "
                       "store the linear renders as float32 .npy (H, W, 4) BGRA instead")
    hdr = _png_header(path)
    if hdr is not None and hdr[2] == 16 and hdr[3] in (2, 4, 6):
        return _read_png16_color(path, hdr[0], hdr[1], hdr[3], hdr[4])
    from PIL import Image
    with Image.open(path) as im:
        im.load()
        mode = im.mode
        if mode == "1":
            return np.asarray(im.convert("L"))
        if mode in ("L", "F"):
            return np.asarray(im).copy()
        if mode in ("I;16", "I;16B", "I;16L", "I"):
            a = np.asarray(im)
            if mode == "I" and (a.min() < 0 or a.max() > 65535):
                raise ImageFormatError(f"{path}: 32-bit integer image")
            return a.astype(np.uint16)
        if mode == "LA":
            a = np.asarray(im)
            g, al = a[..., 0], a[..., 1]
            return np.stack([g, g, g, al], axis=-1)
        if mode == "P":
            im = im.convert("RGB")
            mode = "RGB"
        if mode == "RGB":
            return np.ascontiguousarray(np.asarray(im)[..., ::-1])
        if mode == "RGBA":
            return np.ascontiguousarray(np.asarray(im)[..., [2, 1, 0, 3]])
        raise ImageFormatError(f"{path}: unsupported image mode {mode!r}")


def bgr_to_rgb(img):
    """cv2.cvtColor(img, cv2.COLOR_BGR2RGB) (and COLOR_RGB2BGR): the channel order reversed."""
    if img.ndim != 3 or img.shape[2] != 3:
        raise ImageFormatError(f"BGR <-> RGB needs (H, W, 3) images, got {img.shape}")
    return np.ascontiguousarray(img[..., ::-1])


def bgr_to_gray(img):
    """cv2.cvtColor(img, cv2.COLOR_BGR2GRAY) on float32 (..., H, W, 3) BGR images (see the module
    docstring for the arithmetic)."""
    if img.dtype != np.float32 or img.shape[-1] != 3:
        raise ImageFormatError(f"BGR -> grey expects float32 (..., 3) images, got {img.dtype} {img.shape}")
    cb, cg, cr = (np.float64(c) for c in GRAY_COEFFS_BGR)
    b, g, r = (img[..., k].astype(np.float64) for k in range(3))
    t = (b * cb).astype(np.float32).astype(np.float64)
    t = (g * cg + t).astype(np.float32).astype(np.float64)
    return (r * cr + t).astype(np.float32)


def imwrite(path, img):
    """``cv2.imwrite(path, img)`` for the reference's predictions: uint8 / uint16 (H, W), (H, W, 1)
    or (H, W, 3) BGR arrays -> a PNG holding the same samples (colour stored as RGB, as OpenCV
    does)."""
    from PIL import Image
    a = np.asarray(img)
    if a.ndim == 3 and a.shape[2] == 1:
        a = a[..., 0]
    if a.ndim == 2:
        if a.dtype == np.uint8:
            Image.fromarray(a).save(path)
        elif a.dtype == np.uint16:
            Image.fromarray(a).save(path)
        else:
            raise ImageFormatError(f"imwrite: {a.dtype} grey images are not supported")
        return
    if a.ndim == 3 and a.shape[2] == 3 and a.dtype == np.uint8:
        Image.fromarray(np.ascontiguousarray(a[..., ::-1])).save(path)
        return
    raise ImageFormatError(f"imwrite: unsupported array {a.dtype} {a.shape}")
