"""f4 video I/O: the C driver's YUV4MPEG2 module (host/y4m.c) on CPU, and the
driver end to end on a Y4M clip (GPU)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "phase-based-motion-manipulation_amd")
LIB = os.path.join(PKG, "lib", "liby4m.so")
CLI = os.path.join(PKG, "bin", "mm_cli")


class Info(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("fps_num", ctypes.c_int),
                ("fps_den", ctypes.c_int), ("aspect_num", ctypes.c_int),
                ("aspect_den", ctypes.c_int), ("chroma", ctypes.c_int), ("interlace", ctypes.c_char)]


@pytest.fixture(scope="module")
def y4m():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", PKG, "lib/liby4m.so"])
    L = ctypes.CDLL(LIB)
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    L.y4m_read_header.argtypes = [ctypes.c_void_p, ctypes.POINTER(Info)]
    L.y4m_frame_bytes.restype = ctypes.c_size_t
    L.y4m_frame_bytes.argtypes = [ctypes.POINTER(Info)]
    L.y4m_read_frame.argtypes = [ctypes.c_void_p, ctypes.POINTER(Info), ctypes.c_void_p]
    L.y4m_to_rgba.argtypes = [ctypes.POINTER(Info), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.y4m_from_rgba.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int]
    return L, libc


def write_y4m(path, frames_yuv, W, H, chroma="420", extra=""):
    with open(path, "wb") as f:
        f.write(f"YUV4MPEG2 W{W} H{H} F30000:1001 Ip A1:1 C{chroma}{extra}\n".encode())
        for planes in frames_yuv:
            f.write(b"FRAME\n")
            for p in planes:
                f.write(np.ascontiguousarray(p, np.uint8).tobytes())


def read_all(y4m, path):
    L, libc = y4m
    fp = libc.fopen(path.encode(), b"rb")
    info = Info()
    assert L.y4m_read_header(fp, ctypes.byref(info)) == 0
    nb = L.y4m_frame_bytes(ctypes.byref(info))
    frames = []
    while True:
        buf = np.empty(nb, np.uint8)
        r = L.y4m_read_frame(fp, ctypes.byref(info), buf.ctypes.data)
        if r != 1:
            assert r == 0
            break
        rgba = np.empty((info.height, info.width, 4), np.uint8)
        L.y4m_to_rgba(ctypes.byref(info), buf.ctypes.data, rgba.ctypes.data, 0)
        frames.append(rgba)
    libc.fclose(fp)
    return info, frames


def bt601_to_rgb(Y, Cb, Cr):
    y = (Y.astype(np.float64) - 16) * 255 / 219
    cb = (Cb.astype(np.float64) - 128) * 255 / 224
    cr = (Cr.astype(np.float64) - 128) * 255 / 224
    rgb = np.stack([y + 1.402 * cr, y - 0.344136 * cb - 0.714136 * cr, y + 1.772 * cb], -1)
    return np.clip(np.floor(rgb + 0.5), 0, 255)


def test_header_and_420_decode(y4m, tmp_path):
    W, H = 22, 14
    rng = np.random.default_rng(1)
    Y = rng.integers(16, 236, (H, W))
    Cb = rng.integers(16, 241, (H // 2, W // 2))
    Cr = rng.integers(16, 241, (H // 2, W // 2))
    p = str(tmp_path / "a.y4m")
    write_y4m(p, [(Y, Cb, Cr)] * 2, W, H, "420jpeg", " XYSCSS=420JPEG")
    info, fr = read_all(y4m, p)
    assert (info.width, info.height, info.fps_num, info.fps_den, info.chroma) == (W, H, 30000, 1001, 0)
    assert len(fr) == 2
    ref = bt601_to_rgb(Y, np.repeat(np.repeat(Cb, 2, 0), 2, 1), np.repeat(np.repeat(Cr, 2, 0), 2, 1))
    assert np.abs(fr[0][..., :3].astype(int) - ref).max() <= 1
    assert np.all(fr[0][..., 3] == 255)


def test_444_round_trip_and_mono(y4m, tmp_path):
    L, _ = y4m
    W, H = 32, 16
    rgba = O.synth_frame(W, H, 3)
    planes = np.empty(3 * W * H, np.uint8)
    L.y4m_from_rgba(W, H, rgba.ctypes.data, planes.ctypes.data, 0)
    p = str(tmp_path / "b.y4m")
    write_y4m(p, [planes.reshape(3, H, W)], W, H, "444")
    _, fr = read_all(y4m, p)
    assert np.abs(fr[0].astype(int) - rgba.astype(int)).max() <= 2   # limited-range quantisation
    write_y4m(p, [(np.full((H, W), 235),)], W, H, "mono")
    _, fr = read_all(y4m, p)
    assert np.all(fr[0][..., :3] == 255)


@pytest.mark.parametrize("hdr", ["YUV4MPEG2 W8 H8 C422\n", "YUV4MPEG2 W8 H8 C420p10\n",
                                 "YUV4MPEG2 H8 C420\n", "RIFF W8 H8\n"])
def test_rejects_unsupported(y4m, tmp_path, hdr):
    L, libc = y4m
    p = str(tmp_path / "c.y4m")
    open(p, "w").write(hdr)
    fp = libc.fopen(p.encode(), b"rb")
    assert L.y4m_read_header(fp, ctypes.byref(Info())) == -1
    libc.fclose(fp)


@pytest.mark.gpu
@pytest.mark.parametrize("srgb", [False, True])
def test_cli_y4m_matches_binding(y4m, tmp_path, srgb):
    """mm_cli on a Y4M clip == the same decoded frames through the binding
    (--srgb: the clip's 8-bit RGB taken as sRGB-encoded, MM_RGBA8_SRGB)."""
    import mm355
    import torch
    W, H, n = 64, 48, 5
    rng = np.random.default_rng(7)
    clip = []
    for t in range(n):
        Y = (120 + 60 * np.sin((np.arange(W)[None, :] + 0.4 * t) / 5.0) *
             np.cos(np.arange(H)[:, None] / 7.0) + rng.integers(0, 8, (H, W)))
        clip.append((np.clip(Y, 16, 235), np.full((H // 2, W // 2), 120),
                     np.full((H // 2, W // 2), 136)))
    src, dst = str(tmp_path / "in.y4m"), str(tmp_path / "out.y4m")
    write_y4m(src, clip, W, H)
    subprocess.check_call([CLI, "-i", src, "-o", dst, "-n", str(n), "-l", "5", "-s", "10",
                           "-b", "2"] + (["--srgb"] if srgb else []), timeout=120)
    _, frames = read_all(y4m, src)
    _, got = read_all(y4m, dst)
    assert len(got) == n
    h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=10.0))
    dev = torch.from_numpy(np.stack(frames)).cuda()
    out = torch.empty_like(dev)
    h.process_stream(dev, out, n, mm355.RGBA8_SRGB if srgb else mm355.RGBA8)
    torch.cuda.synchronize()
    h.close()
    L, _ = y4m
    info = Info(W, H, 25, 1, 1, 1, 1, b"p")   # 4:4:4 planes of the driver's output
    for k, o in enumerate(out.cpu().numpy()):
        planes = np.empty(3 * W * H, np.uint8)
        L.y4m_from_rgba(W, H, np.ascontiguousarray(o).ctypes.data, planes.ctypes.data, 0)
        rgba = np.empty((H, W, 4), np.uint8)
        L.y4m_to_rgba(ctypes.byref(info), planes.ctypes.data, rgba.ctypes.data, 0)
        assert np.array_equal(rgba, got[k]), k
