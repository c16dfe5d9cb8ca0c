"""mm355 — Python host mirror of the MI355X-native MotionMagnificationProcessor.

The product is the C-ABI library ``lib/libmm355.so`` (include/mm.h) whose HIP
kernels do all the work.  This module binds it with ctypes and mirrors the
reference Unity component's operator surface
(Assets/Scripts/MotionMagnificationProcessor.cs) so a user of the reference
finds the same names, argument meaning and error behaviour:

    proc = MotionMagnificationProcessor(width, height, pyramid_levels=5,
                                        phase_scale=25.0)
    proc.Start()                       # .cs:90  -> mm_create
    proc.OnRenderImage(src, dst)       # .cs:101 -> mm_process
    proc.phase_scale = 10.0; proc.OnValidate()   # .cs:78 -> mm_set_params
    proc.OnDestroy()                   # .cs:96  -> mm_destroy

There is no CPU fallback.  If the library or a gfx950 device is missing,
construction/Start raises ``MMError`` — loudly, never silently.
"""
from .binding import (MMError, lib, load_library, LIB_PATH, RGBA8, RGBA32F, RGBA16F, RGBA8_SRGB,
                      FORMAT_BPP, frame_bytes,
                      EDGE_REPEAT, EDGE_CLAMP, MODE_PYRAMID, MODE_STANDARD, MODE_STEERABLE,
                      FILTER_DIFF, FILTER_IIR, Params, Handle,
                      abi_symbols, resample_table, strerror)
from .processor import MotionMagnificationProcessor
from .stream import ShardedStream, shard_range
from .ring import Ring, new_ring_id, ring_lib

__all__ = ["MMError", "lib", "load_library", "LIB_PATH", "RGBA8", "RGBA32F", "RGBA16F",
           "RGBA8_SRGB", "FORMAT_BPP", "frame_bytes",
           "EDGE_REPEAT", "EDGE_CLAMP", "MODE_PYRAMID", "MODE_STANDARD", "MODE_STEERABLE",
           "FILTER_DIFF", "FILTER_IIR", "Params", "Handle", "abi_symbols",
           "resample_table", "strerror", "MotionMagnificationProcessor",
           "ShardedStream", "shard_range", "Ring", "new_ring_id", "ring_lib"]
