"""Mirror of the reference Unity component ``MotionMagnificationProcessor``
(Assets/Scripts/MotionMagnificationProcessor.cs) on top of the C-ABI.

Field names follow the reference's serialized inspector fields (.cs:7-43) in
snake_case; methods keep the reference's Unity callback names.
"""
import numpy as np

from .binding import (EDGE_REPEAT, FILTER_DIFF, MODE_PYRAMID, MODE_STANDARD, MODE_STEERABLE,
                      RGBA8, RGBA8_SRGB, RGBA16F, RGBA32F, Handle, MMError, Params)


def _fmt_of(frame, srgb=False):
    """Frame format from the dtype: uint8 UNORM (or sRGB-encoded with srgb),
    float16 (linear half, the HDR camera target), float32."""
    dt = str(getattr(frame, "dtype", ""))
    if dt.endswith("uint8"):
        return RGBA8_SRGB if srgb else RGBA8
    if dt.endswith("float16"):
        return RGBA16F
    if dt.endswith("float32"):
        return RGBA32F
    raise MMError(-1, f"frame dtype {dt} (want uint8, float16 or float32 RGBA)")


def _is_device(frame):
    return bool(getattr(frame, "is_cuda", False))


class MotionMagnificationProcessor:
    """[RequireComponent(typeof(Camera))] class MotionMagnificationProcessor (.cs:4-5).

    ``width``/``height`` play the role of Screen.width/height read in
    InitializeProcessor (.cs:298-299): geometry is frozen at Start().
    """

    def __init__(self, width, height, *, apply_motion_magnification=True,
                 show_magnitude=False, show_phase=False, use_pyramid_decomposition=True,
                 pyramid_levels=5, min_frequency=0.05, max_frequency=0.45,
                 phase_scale=10.0, magnitude_threshold=0.01, apply_bandpass_filter=True,
                 low_frequency_cutoff=0.05, high_frequency_cutoff=0.4, filter_steepness=3.0,
                 motion_sensitivity=1.5, enhance_edges=True, edge_enhancement=0.8,
                 edge_mode=EDGE_REPEAT, orientations=1, temporal_filter=FILTER_DIFF,
                 iir_low=None, iir_high=None, srgb=False, device=0):
        self.width, self.height, self.device = width, height, device
        # 8-bit frames are sRGB-encoded render targets under Unity's Linear colour
        # space (ProjectSettings/ProjectSettings.asset:50): decoded to linear light
        # on read and encoded on write (MM_RGBA8_SRGB); False: UNORM bytes
        self.srgb = srgb
        self.apply_motion_magnification = apply_motion_magnification  # .cs:12
        self.show_magnitude = show_magnitude                          # .cs:13
        self.show_phase = show_phase                                  # .cs:14
        self.use_pyramid_decomposition = use_pyramid_decomposition    # .cs:18
        self.pyramid_levels = pyramid_levels                          # .cs:19
        self.min_frequency = min_frequency                            # .cs:20
        self.max_frequency = max_frequency                            # .cs:21
        self.phase_scale = phase_scale                                # .cs:29
        self.magnitude_threshold = magnitude_threshold                # .cs:30
        self.apply_bandpass_filter = apply_bandpass_filter            # .cs:35
        self.low_frequency_cutoff = low_frequency_cutoff              # .cs:36
        self.high_frequency_cutoff = high_frequency_cutoff            # .cs:37
        self.filter_steepness = filter_steepness                      # .cs:38
        self.motion_sensitivity = motion_sensitivity                  # .cs:41
        self.enhance_edges = enhance_edges                            # .cs:42
        self.edge_enhancement = edge_enhancement                      # .cs:43
        self.edge_mode = edge_mode
        # steerable extension (no reference counterpart):
        # orientations 4/6/8 with the pyramid switch on select MM_MODE_STEERABLE;
        # iir_low/iir_high None keep mm_params_default's coefficients
        self.orientations = orientations
        self.temporal_filter = temporal_filter
        self.iir_low, self.iir_high = iir_low, iir_high
        self._handle = None

    # -- reference lifecycle -------------------------------------------------
    def _params(self):
        # usePyramidDecomposition selects ProcessFrameWithPyramidDecomposition or
        # ProcessFrameWithStandardMagnification (.cs:128-135)
        mode = MODE_PYRAMID if self.use_pyramid_decomposition else MODE_STANDARD
        steer = {}
        if self.use_pyramid_decomposition and self.orientations != 1:
            mode = MODE_STEERABLE
            steer = dict(orientations=self.orientations, temporal_filter=self.temporal_filter)
            if self.iir_low is not None:
                steer["iir_low"] = self.iir_low
            if self.iir_high is not None:
                steer["iir_high"] = self.iir_high
        return Params.make(levels=self.pyramid_levels, min_freq=self.min_frequency,
                           max_freq=self.max_frequency, phase_scale=self.phase_scale,
                           magnitude_threshold=self.magnitude_threshold,
                           edge_mode=self.edge_mode,
                           apply_magnification=self.apply_motion_magnification, mode=mode,
                           apply_bandpass_filter=self.apply_bandpass_filter,
                           low_frequency_cutoff=self.low_frequency_cutoff,
                           high_frequency_cutoff=self.high_frequency_cutoff,
                           filter_steepness=self.filter_steepness,
                           motion_sensitivity=self.motion_sensitivity,
                           enhance_edges=self.enhance_edges,
                           edge_enhancement=self.edge_enhancement,
                           # showMagnitude / showPhase: ProcessDebugView (.cs:119-123)
                           show_magnitude=self.show_magnitude, show_phase=self.show_phase,
                           **steer)

    def Start(self):
        """Start -> InitializeProcessor (.cs:90-94, :289-342). Raises on failure."""
        self._handle = Handle(self.width, self.height, self._params(), self.device)
        return self

    def OnValidate(self):
        """OnValidate (.cs:78-88): push edited fields; effective next frame."""
        if self._handle is not None:
            self._handle.set_params(self._params())

    def OnRenderImage(self, source, destination):
        """OnRenderImage (.cs:101-143). source/destination: [H, W, 4] uint8,
        float16 or float32, both torch CUDA tensors (async on torch's current
        stream) or both host numpy arrays (synchronous)."""
        if self._handle is None:                       # !isInitialized -> Blit (.cs:103-107)
            destination[...] = source
            return
        fmt = _fmt_of(source, self.srgb)
        if _fmt_of(destination, self.srgb) != fmt:
            raise MMError(-1, "source/destination formats differ")
        on_dev = _is_device(source)
        if on_dev != _is_device(destination):
            raise MMError(-1, "source and destination must both be device or host")
        if not on_dev:
            if not (source.flags.c_contiguous and destination.flags.c_contiguous):
                raise MMError(-1, "frames must be C-contiguous")
        elif not (source.is_contiguous() and destination.is_contiguous()):
            raise MMError(-1, "frames must be contiguous")
        stream = None
        if on_dev:   # order after whatever produced `source` on torch's current stream
            import torch
            stream = torch.cuda.current_stream(source.device).cuda_stream
        self._handle.process(source, destination, fmt, on_device=on_dev, stream=stream)

    def OnDestroy(self):
        """OnDestroy -> ReleaseResources (.cs:96-99, :344-356)."""
        if self._handle is not None:
            self._handle.close()
            self._handle = None

    # -- extras ---------------------------------------------------------------
    def reset(self):
        """isFirstFrame = true (.cs:75): next frame passes through."""
        self._handle.reset()

    @property
    def handle(self):
        return self._handle

    @property
    def padded_size(self):
        return self._handle.N if self._handle else None


def host_frames(n, h, w, fmt):
    dt = {RGBA8: np.uint8, RGBA8_SRGB: np.uint8, RGBA16F: np.float16}.get(fmt, np.float32)
    return np.zeros((n, h, w, 4), dt)
