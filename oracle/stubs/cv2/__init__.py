"""Oracle-only stand-in for OpenCV (absent from the image; the reference imports cv2 at module load,
utils/__init__.py:22) — TEST INFRASTRUCTURE ONLY.

Nothing on the detector's compute path calls cv2. The training augmentations do (data/augment.py: RandomHSV
:1344-1378, RandomPerspective.affine_transform :1016-1077), so the few functions they call are restated here in
numpy from OpenCV 4.x's published algorithms, so that the reference's own transform code can be run to make the
augmentation fixtures (oracle/gen_golden.py `augment`). The reference pins no OpenCV version
(pyproject.toml: opencv-python>=4.6.0) and OpenCV itself is not installed: these restatements are PARITY
UNPINNED against real OpenCV; they pin the reference's arithmetic around them (RNG order, matrices, labels).

  cvtColor BGR2HSV (8U):  imgproc color_hsv: hsv_shift 12, sdiv_table / hdiv_table180 (cvRound of 255<<12 / i,
                          180<<12 / 6i), s = (diff*sdiv[v] + 2^11) >> 12, h selected by the max channel
                          (r first, then g), h = (h*hdiv[diff] + 2^11) >> 12, + 180 if negative.
  cvtColor HSV2BGR (8U):  u8 -> float (h, s/255, v/255), HSV2RGB_native in float32 (hscale 6.f/180, sector
                          table), saturate_cast<uchar>(x*255.f) (round half to even, clamp).
  warpAffine (INTER_LINEAR, BORDER_CONSTANT, 8U): the 2x3 matrix in double, inverted as invertAffineTransform;
                          fixed-point coordinates AB_BITS 10 / INTER_BITS 5 (adelta = cvRound(M0*x*1024),
                          X0 = cvRound((M1*y + M2)*1024) + 16, X = (X0 + adelta) >> 5); bilinear weights
                          (32-fx)(32-fy)*32 etc. (INTER_REMAP_COEF_BITS 15), (sum + 2^14) >> 15; neighbours outside
                          the source take borderValue, a sample with no neighbour inside is borderValue.
  getRotationMatrix2D:    a = angle * (pi/180), alpha = cos(a)*scale, beta = sin(a)*scale, double (libm).
"""
import math

import numpy as np

__version__ = "0.0.0-oracle-stub"

COLOR_BGR2HSV = 40
COLOR_HSV2BGR = 54
INTER_LINEAR = 1
BORDER_CONSTANT = 0


def setNumThreads(n):  # noqa: N802 (OpenCV naming)
    return None


def __getattr__(name):
    return 0


_HSV_SHIFT = 12
_SDIV = np.array([0] + [int(np.rint((255 << _HSV_SHIFT) / float(i))) for i in range(1, 256)], dtype=np.int64)
_HDIV180 = np.array([0] + [int(np.rint((180 << _HSV_SHIFT) / (6.0 * i))) for i in range(1, 256)], dtype=np.int64)


def bgr2hsv_u8(img):
    b, g, r = (img[..., k].astype(np.int64) for k in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    s = (diff * _SDIV[v] + (1 << (_HSV_SHIFT - 1))) >> _HSV_SHIFT
    h = np.where(v == r, g - b, np.where(v == g, b - r + 2 * diff, r - g + 4 * diff))
    h = (h * _HDIV180[diff] + (1 << (_HSV_SHIFT - 1))) >> _HSV_SHIFT
    h = np.where(h < 0, h + 180, h)
    return np.stack([h, s, v], -1).astype(np.uint8)


_SECTOR = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])


def hsv2bgr_u8(img):
    f32 = np.float32
    h = img[..., 0].astype(f32)
    s = img[..., 1].astype(f32) * (f32(1.0) / f32(255.0))
    v = img[..., 2].astype(f32) * (f32(1.0) / f32(255.0))
    hs = h * (f32(6.0) / f32(180.0))
    hs = np.fmod(hs, f32(6.0))
    sector = np.floor(hs).astype(np.int64)
    hf = (hs - sector.astype(f32)).astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    hf = np.where(bad, f32(0.0), hf)
    one = f32(1.0)
    tab = np.stack([v, v * (one - s), v * (one - s * hf), v * (one - s * (one - hf))], -1).astype(f32)
    idx = _SECTOR[sector]  # (..., 3) -> b, g, r
    bgr = np.take_along_axis(tab, idx, -1)
    bgr = np.where((s == 0)[..., None], v[..., None], bgr).astype(f32)
    out = np.rint(bgr * f32(255.0))
    return np.clip(out, 0, 255).astype(np.uint8)


def cvtColor(img, code, dst=None):  # noqa: N802
    if code == COLOR_BGR2HSV:
        out = bgr2hsv_u8(img)
    elif code == COLOR_HSV2BGR:
        out = hsv2bgr_u8(img)
    else:
        raise NotImplementedError(f"cv2 stub: cvtColor code {code}")
    if dst is not None:
        dst[...] = out
        return dst
    return out


def split(img):
    return tuple(np.ascontiguousarray(img[..., k]) for k in range(img.shape[-1]))


def merge(chs):
    return np.stack(chs, -1)


def LUT(src, lut):  # noqa: N802
    return np.asarray(lut)[src]


def getRotationMatrix2D(center, angle, scale):  # noqa: N802
    a = angle * (math.pi / 180)  # angle *= CV_PI/180
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    cx, cy = center
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy], [-beta, alpha, beta * cx + (1 - alpha) * cy]],
                    dtype=np.float64)


def warp_affine_tables(M, dsize):
    """Fixed-point source coordinates of cv::warpAffine (INTER_LINEAR): per destination column adelta/bdelta and per
    row X0/Y0 (int64), with the inverse of the 2x3 matrix M computed in double as warpAffine does."""
    m = np.asarray(M, dtype=np.float64).reshape(6).copy()
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = m[4] * D, m[0] * D
    m[0], m[4] = A11, A22
    m[1] *= -D
    m[3] *= -D
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    W, H = dsize
    xs = np.arange(W, dtype=np.float64)
    ys = np.arange(H, dtype=np.float64)
    adelta = np.rint(m[0] * xs * 1024).astype(np.int64)
    bdelta = np.rint(m[3] * xs * 1024).astype(np.int64)
    X0 = np.rint((m[1] * ys + m[2]) * 1024).astype(np.int64) + 16
    Y0 = np.rint((m[4] * ys + m[5]) * 1024).astype(np.int64) + 16
    return adelta, bdelta, X0, Y0


def warpAffine(img, M, dsize, borderValue=(0, 0, 0), **kw):  # noqa: N802
    if kw.get("flags", INTER_LINEAR) != INTER_LINEAR or img.dtype != np.uint8 or img.ndim != 3:
        raise NotImplementedError("cv2 stub: warpAffine covers 8U 3-channel INTER_LINEAR only")
    adelta, bdelta, X0, Y0 = warp_affine_tables(M, dsize)
    X = (X0[:, None] + adelta[None, :]) >> 5
    Y = (Y0[:, None] + bdelta[None, :]) >> 5
    sx, sy, fx, fy = X >> 5, Y >> 5, X & 31, Y & 31
    Hs, Ws = img.shape[:2]
    cval = np.asarray(borderValue[:3], dtype=np.int64)
    acc = np.zeros(sx.shape + (3,), dtype=np.int64)
    for dy in (0, 1):
        for dx in (0, 1):
            wgt = ((32 - fx) if dx == 0 else fx) * ((32 - fy) if dy == 0 else fy) * 32
            yy, xx = sy + dy, sx + dx
            ok = (yy >= 0) & (yy < Hs) & (xx >= 0) & (xx < Ws)
            v = img[np.clip(yy, 0, Hs - 1), np.clip(xx, 0, Ws - 1)].astype(np.int64)
            v = np.where(ok[..., None], v, cval)
            acc += v * wgt[..., None]
    out = (acc + (1 << 14)) >> 15
    none = (sx >= Ws) | (sx + 1 < 0) | (sy >= Hs) | (sy + 1 < 0)
    out = np.where(none[..., None], cval, out)
    return np.clip(out, 0, 255).astype(np.uint8)
