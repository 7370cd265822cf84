"""PNG encoding for the evaluation-view fixtures and tests (test infrastructure): ``encode_png`` writes
non-interlaced PNGs whose scanlines use every filter type; ``bgr`` is what cv2.imread
(IMREAD_UNCHANGED) returns for a file holding given grey / grey + alpha / RGB / RGBA samples."""
import numpy as np


def _png_chunk(kind, data):
    import struct
    import zlib
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def encode_png(arr, depth):
    """PNG bytes of (H, W[, C]) samples (grey / grey+alpha / RGB / RGBA, 8 or 16 bits), non-interlaced,
    row y filtered with type y mod 5 (None, Sub, Up, Average, Paeth) so that a reader's unfiltering
    is exercised.  Encoding reads only raw neighbours, so each row is vectorised."""
    import struct
    import zlib
    a = np.asarray(arr)
    H, W = a.shape[:2]
    C = 1 if a.ndim == 2 else a.shape[2]
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[C]
    raw = np.ascontiguousarray(a.astype(">u2" if depth == 16 else np.uint8)).view(np.uint8).reshape(H, -1)
    raw = raw.astype(np.int32)
    bpp = C * depth // 8
    rows, prev = [], np.zeros(raw.shape[1], np.int32)
    for y in range(H):
        x = raw[y]
        left = np.concatenate([np.zeros(bpp, np.int32), x[:-bpp]])
        upl = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        ft = y % 5
        if ft == 0:
            f = x
        elif ft == 1:
            f = x - left
        elif ft == 2:
            f = x - prev
        elif ft == 3:
            f = x - ((left + prev) >> 1)
        else:
            p = left + prev - upl
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - upl)
            f = x - np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, upl))
        rows.append(bytes([ft]) + (f & 255).astype(np.uint8).tobytes())
        prev = x
    return (b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, 0))
            + _png_chunk(b"IDAT", zlib.compress(b"".join(rows))) + _png_chunk(b"IEND", b""))


def bgr(samples):
    """What cv2.imread returns for a file holding (H, W[, C]) grey / GA / RGB / RGBA samples."""
    a = np.asarray(samples)
    if a.ndim == 2:
        return a.copy()
    C = a.shape[2]
    if C == 2:
        return np.stack([a[..., 0], a[..., 0], a[..., 0], a[..., 1]], axis=-1)
    if C == 3:
        return np.ascontiguousarray(a[..., ::-1])
    return np.ascontiguousarray(a[..., [2, 1, 0, 3]])
