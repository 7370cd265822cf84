"""On-disk formats the hot path reads -- mirror of the reference's data/datasets.py (Event :14-373,
PosedImage :376-712, CameraPose :715-758) with the same file names, keys and classmethods:

* ``camera_calibration.npz`` (intrinsics, distortion, image size, bayer_pattern, contrast
  thresholds, refractory period, pixel-bandwidth constants) -- numpy, no pickles;
* ``raw_events.npz`` -- position (n, 2) uint16, timestamp (n) i64 ns, polarity (n) bool
  (scripts/preprocess_esim.py:340-345);
* ``events.pt`` -- the queued events (position, start_ts, end_ts, num_pos, num_neg[, channel_idx]),
  built from ``raw_events.npz`` on the first construction and cached (datasets.py:43-55);
* ``max_refractory_period.pt`` -- a scalar tensor, extracted from the raw events and cached the same
  way (models/event_generation_params.py:135-149);
* ``camera_poses.npz`` -- T_wc_position (C, 3), T_wc_orientation (C, 4) XYZW, T_wc_timestamp (C) ns;
* ``views/transforms_{train,val,test}.json`` + image files + ``renderer_params.npz`` -- the evaluation
  views (``PosedImage``; images read by ``utils/image_io`` in OpenCV's conventions).

The build path's per-event work (the reference's per-pixel deque loops, colorization and
undistortion) runs on the GPU in libden.so (den_queue_raw_events, den_max_refractory_period,
den_colorize_events, den_undistort_events); there is no CPU fallback.  Cached tensors are loaded
with ``torch.load(weights_only=True)``.
"""
import glob
import json
import math
import os

import numpy as np
import torch

from .. import _native
from ..utils import image_io
from ..utils.easydict import EasyDict


def _atomic_torch_save(obj, path):
    """torch.save to a per-process temporary file in the same directory, then os.replace onto the final
    name: DDP ranks that each build a missing cache never expose a half-written file to one another."""
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _device():
    """The GPU the build-path kernels run on (the current HIP device)."""
    if not torch.cuda.is_available():
        raise _native.DenError("building events.pt / max_refractory_period.pt from raw_events.npz needs a HIP "
                               "device (libden.so; there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


class Event(torch.utils.data.Dataset):
    RAW_EVENTS_FILENAME = "raw_events.npz"
    TF_EVENTS_FILENAME = "events.pt"
    CAMERA_CALIBRATION_FILENAME = "camera_calibration.npz"
    MAX_REFRACTORY_PERIOD_FILENAME = "max_refractory_period.pt"
    RAW_EVENT_POSITION_KEY = "position"
    RAW_EVENT_TIMESTAMP_KEY = "timestamp"
    RAW_EVENT_POLARITY_KEY = "polarity"
    IMG_HEIGHT_KEY = "img_height"
    IMG_WIDTH_KEY = "img_width"
    DISTORTION_MODEL_KEY = "distortion_model"
    DISTORTION_PARAMS_KEY = "distortion_params"
    INTRINSICS_KEY = "intrinsics"
    BAYER_PATTERN_KEY = "bayer_pattern"
    NULL_BAYER_PATTERN = ""
    BAYER_PATTERN_LEN = 4
    COLOR_CHANNEL_NAME_TO_INDEX = {"R": 0, "G": 1, "B": 2}

    def __init__(self, root_directory, permutation_seed=None):
        super().__init__()
        # datasets.py:43-55: the cached transformed events, else queue + colorize + undistort + cache
        self.events = self.load_transformed_events(root_directory)
        if self.events is None:
            camera_calibration = self.load_camera_calibration(root_directory)
            events = self.queue_raw_events(root_directory, camera_calibration)
            events = self.colorize_events(events, camera_calibration)
            events = self.undistort_events(events, camera_calibration)
            self.events = EasyDict({k: v.cpu() for k, v in events.items()})
            self.save_transformed_events(self.events, root_directory)
        if permutation_seed is not None:
            g = torch.Generator()
            g.manual_seed(permutation_seed)
            perm = torch.randperm(len(self.events.position), generator=g)
            for k, v in self.events.items():
                self.events[k] = v[perm]

    @classmethod
    def load_transformed_events(cls, root_directory):
        path = os.path.join(root_directory, cls.TF_EVENTS_FILENAME)
        if not os.path.isfile(path):
            return None
        return EasyDict(torch.load(path, weights_only=True))

    @classmethod
    def save_transformed_events(cls, transformed_events, root_directory):
        _atomic_torch_save(dict(transformed_events), os.path.join(root_directory, cls.TF_EVENTS_FILENAME))

    @classmethod
    def load_raw_events(cls, root_directory):
        return np.load(os.path.join(root_directory, cls.RAW_EVENTS_FILENAME), allow_pickle=False)

    @classmethod
    def load_camera_calibration(cls, root_directory):
        return np.load(os.path.join(root_directory, cls.CAMERA_CALIBRATION_FILENAME), allow_pickle=False)

    @classmethod
    def load_max_refractory_period(cls, root_directory):
        path = os.path.join(root_directory, cls.MAX_REFRACTORY_PERIOD_FILENAME)
        return torch.load(path, weights_only=True) if os.path.isfile(path) else None

    @classmethod
    def save_max_refractory_period(cls, max_refractory_period, root_directory):
        _atomic_torch_save(max_refractory_period, os.path.join(root_directory, cls.MAX_REFRACTORY_PERIOD_FILENAME))

    @classmethod
    def _raw_on_device(cls, raw_events, camera_calibration):
        pos = np.asarray(raw_events[cls.RAW_EVENT_POSITION_KEY])
        ts = np.asarray(raw_events[cls.RAW_EVENT_TIMESTAMP_KEY])
        pol = np.asarray(raw_events[cls.RAW_EVENT_POLARITY_KEY])
        assert len(pos) == len(ts) == len(pol)
        if not np.issubdtype(ts.dtype, np.integer):
            raise _native.DenError(f"raw event timestamps must be integer ns, got {ts.dtype}")
        if pol.dtype != np.bool_ and not np.isin(pol, (0, 1)).all():
            raise _native.DenError("raw event polarities must be boolean (datasets.py:208 casts them to {1, 0})")
        dev = _device()
        # datasets.py:205-208: positions cast to int64, polarities {True, False} -> {1, 0}
        pos_t = torch.from_numpy(pos.astype(np.int64)).to(dev)
        ts_t = torch.from_numpy(ts.astype(np.int64)).to(dev)
        pol_t = torch.from_numpy(pol.astype(bool)).to(dev)
        H = int(camera_calibration[cls.IMG_HEIGHT_KEY])
        W = int(camera_calibration[cls.IMG_WIDTH_KEY])
        return pos_t, ts_t, pol_t, H, W, ts.dtype

    @classmethod
    def extract_max_refractory_period(cls, raw_events, camera_calibration):
        """datasets.py:133-187 on the device (den_max_refractory_period): the minimum event interval
        over the pixels' substreams -> an int64 scalar tensor, or inf (f64) when no pixel has two
        distinct timestamps, as the reference's min over np.int64 intervals from np.array(inf)."""
        pos, ts, _, H, W, _ = cls._raw_on_device(raw_events, camera_calibration)
        mx = _native.max_refractory_period(pos, ts, H, W)
        return torch.tensor(float("inf"), dtype=torch.float64) if mx is None else torch.tensor(mx, dtype=torch.int64)

    @classmethod
    def queue_raw_events(cls, root_directory, camera_calibration):
        """datasets.py:190-284 on the device (den_queue_raw_events): -> EasyDict of position (M,2) i64,
        start_ts, end_ts, num_pos, num_neg (M) in the timestamps' dtype, in input order."""
        raw = cls.load_raw_events(root_directory)
        pos, ts, pol, H, W, ts_dtype = cls._raw_on_device(raw, camera_calibration)
        queued, _ = _native.queue_raw_events(pos, ts, pol, H, W)
        tdt = torch.from_numpy(np.zeros(0, dtype=ts_dtype)).dtype  # np.empty_like(timestamps) (:224-227)
        for k in ("start_ts", "end_ts", "num_pos", "num_neg"):
            queued[k] = queued[k].to(tdt)
        return EasyDict(queued)

    @classmethod
    def colorize_events(cls, events, camera_calibration):
        """datasets.py:287-328: channel_idx (u8) from the bayer pattern (den_colorize_events);
        a monochrome camera ("") keeps the events as they are."""
        bayer_pattern = str(camera_calibration[cls.BAYER_PATTERN_KEY])
        assert len(bayer_pattern) in (len(cls.NULL_BAYER_PATTERN), cls.BAYER_PATTERN_LEN)
        if bayer_pattern == cls.NULL_BAYER_PATTERN:
            return events
        assert set(cls.COLOR_CHANNEL_NAME_TO_INDEX.keys()) == set(bayer_pattern)
        channels = [cls.COLOR_CHANNEL_NAME_TO_INDEX[c] for c in bayer_pattern]
        events.channel_idx = _native.colorize_events(events.position, channels)
        return events

    @classmethod
    def undistort_events(cls, events, camera_calibration):
        """datasets.py:331-364 (den_undistort_events): positions to the default dtype, then the
        plumb_bob / equidistant undistortion with P = intrinsics when distortion parameters exist
        (OpenCV's iterations restated; parity unpinned, OpenCV is not in this image)."""
        params = np.asarray(camera_calibration[cls.DISTORTION_PARAMS_KEY]) \
            if cls.DISTORTION_PARAMS_KEY in camera_calibration else np.zeros(0, dtype=np.float32)
        assert len(params) in (0, 4)
        model = str(camera_calibration[cls.DISTORTION_MODEL_KEY]) if len(params) else None
        intrinsics = camera_calibration[cls.INTRINSICS_KEY] if len(params) else np.eye(3, dtype=np.float32)
        pos = events.position
        if pos.dtype != torch.int64:
            raise _native.DenError("undistort_events expects the queued int64 positions")
        out = _native.undistort_events(pos, model, intrinsics, params)
        events.position = out.to(torch.get_default_dtype())
        return events

    def __getitem__(self, index):
        return {k: v[index] for k, v in self.events.items()}

    def __len__(self):
        return len(self.events.position)


def _require(cond, msg):
    """The reference's input checks are asserts (datasets.py:592-605); the same exception type."""
    if not cond:
        raise AssertionError(msg)


class PosedImage(torch.utils.data.Dataset):
    """The evaluation views (data/datasets.py:376-712): ``views/transforms_<stage>.json`` (frames with
    ``file_path``, ``transform_matrix`` in the OpenGL camera convention, optional ``exposure_time`` /
    ``gain``; ``camera_angle_x`` or ``intrinsics``; optional ``bit_depth``), the image files next to
    it, ``renderer_params.npz`` for synthetic renders.  ``posed_imgs`` holds sample_id (N, 16) i64
    (Unicode code points, space padded), img (N, [3,] H, W) f32 normalised intensities (RGB for a
    Bayer sensor, else grey), T_wc_position (N, 3), T_wc_orientation (N, 3, 3) (the common camera
    convention), intrinsics (3, 3), exposure_time / gain (N) when given; ``min_normalized_pixel_value``
    / ``max_normalized_pixel_value`` bound the image values.

    Images are read without OpenCV (``utils/image_io.imread_unchanged``: OpenCV's sample types and
    channel order); the transforms below are the reference's arithmetic in the same dtypes --
    alpha compositing in f64 (display) or f32 (linear), the f32 cast, BGR -> RGB / grey, the
    half-level quantisation normalisation -- so quantised views come out bit-identical.  One deviation
    in numpy promotion: the reference (numpy 1.24, environment.yml:15) adds ``log_eps`` to linear
    renders as a 0-d float64 array, which value-based casting performs in float32; so does this
    class, where numpy >= 2 would promote to float64."""
    STAGES = ("train", "val", "test")
    NORMALIZED_SAMPLE_ID_CHAR_LEN = 16
    ACCEPTED_NUM_IMG_CHANNELS = (1, 3, 4)  # ie. Gray, BGR, BGRA format
    T_COPENGL_CCOMMON_ORIENTATION = np.array([[1, 0, 0], [0, -1, 0], [0, 0, -1]])
    POSED_IMG_FOLDER_NAME = "views"
    STAGE_TRANSFORMS_FILENAME_FORMAT_STR = "transforms_{}.json"
    HORIZONTAL_FOV_KEY = "camera_angle_x"
    INTRINSICS_KEY = "intrinsics"
    BIT_DEPTH_KEY = "bit_depth"
    IMG_METADATA_KEY = "frames"
    IMG_PATH_KEY = "file_path"
    IMG_EXPOSURE_TIME_KEY = "exposure_time"
    IMG_GAIN_KEY = "gain"
    IMG_POSE_KEY = "transform_matrix"
    RENDERER_PARAMS_FILENAME = "renderer_params.npz"
    INTERM_COLOR_SPACE_KEY = "interm_color_space"
    LOG_EPS_KEY = "log_eps"
    BAYER_PATTERN_KEY = "bayer_pattern"
    NULL_BAYER_PATTERN = ""

    def __init__(self, root_directory, stage, permutation_seed, alpha_over_white_bg=False):
        super().__init__()
        assert stage in self.STAGES
        stage_transforms = self.load_stage_transforms(root_directory, stage)
        renderer_params = self.load_renderer_params(root_directory)
        camera_calibration = Event.load_camera_calibration(root_directory)
        self.posed_imgs = self.load_posed_imgs(root_directory, stage_transforms)
        self.posed_imgs = self.transform_img(self.posed_imgs, alpha_over_white_bg, stage_transforms, renderer_params,
                                             camera_calibration)
        self.posed_imgs = self.transform_pose(self.posed_imgs)
        if permutation_seed is None:  # datasets.py:425-434 (tensor_ops.randperm_manual_seed)
            return
        g = torch.Generator()
        g.manual_seed(permutation_seed)
        perm = torch.randperm(len(self.posed_imgs.img), generator=g)
        for k, v in self.posed_imgs.items():
            if k != "intrinsics":
                self.posed_imgs[k] = v[perm]

    @classmethod
    def posed_img_folder_path(cls, root_directory):
        """``views`` in the dataset directory or one level above it (:435-444); None if neither."""
        for path in (os.path.join(root_directory, cls.POSED_IMG_FOLDER_NAME),
                     os.path.join(root_directory, "..", cls.POSED_IMG_FOLDER_NAME)):
            if os.path.isdir(path):
                return path
        return None

    @classmethod
    def load_stage_transforms(cls, root_directory, stage):
        folder = cls.posed_img_folder_path(root_directory)
        if folder is None:
            raise FileNotFoundError(f"no {cls.POSED_IMG_FOLDER_NAME}/ folder in or above {root_directory}")
        with open(os.path.join(folder, cls.STAGE_TRANSFORMS_FILENAME_FORMAT_STR.format(stage))) as f:
            return json.load(f)

    @classmethod
    def load_renderer_params(cls, root_directory):
        path = os.path.join(root_directory, cls.RENDERER_PARAMS_FILENAME)
        return np.load(path, allow_pickle=False) if os.path.isfile(path) else None

    @classmethod
    def load_posed_imgs(cls, root_directory, stage_transforms):
        """:469-547: per frame the space-padded id as code points, the image as read, the pose's
        translation / rotation; then the intrinsics from ``camera_angle_x`` (principal point at the
        pixel-centre convention W / 2 - 0.5) or ``intrinsics``."""
        posed = EasyDict(sample_id=[], img=[], T_wc_position=[], T_wc_orientation=[], intrinsics=None)
        frames = stage_transforms[cls.IMG_METADATA_KEY]
        if len(frames) > 0:
            if cls.IMG_EXPOSURE_TIME_KEY in frames[0].keys():
                posed.exposure_time = []
            if cls.IMG_GAIN_KEY in frames[0].keys():
                posed.gain = []
        folder = cls.posed_img_folder_path(root_directory)
        for meta in frames:
            sample_id = os.path.basename(meta[cls.IMG_PATH_KEY])
            posed.sample_id.append(np.asarray(list(map(ord, sample_id.ljust(cls.NORMALIZED_SAMPLE_ID_CHAR_LEN)))))
            matches = sorted(glob.glob(os.path.join(folder, meta[cls.IMG_PATH_KEY] + ".*")))
            if not matches:
                raise FileNotFoundError(f"no image file for {meta[cls.IMG_PATH_KEY]!r} in {folder}")
            posed.img.append(image_io.imread_unchanged(matches[0]))
            T_wc = np.array(meta[cls.IMG_POSE_KEY])
            posed.T_wc_position.append(T_wc[:3, 3])
            posed.T_wc_orientation.append(T_wc[:3, :3])
            if cls.IMG_EXPOSURE_TIME_KEY in meta.keys():
                posed.exposure_time.append(meta[cls.IMG_EXPOSURE_TIME_KEY])
            if cls.IMG_GAIN_KEY in meta.keys():
                posed.gain.append(meta[cls.IMG_GAIN_KEY])
        for k, v in posed.items():
            if k != "intrinsics":
                posed[k] = np.stack(v, axis=0)
        posed.sample_id = torch.tensor(posed.sample_id)
        assert cls.HORIZONTAL_FOV_KEY in stage_transforms.keys() or cls.INTRINSICS_KEY in stage_transforms.keys()
        if cls.HORIZONTAL_FOV_KEY in stage_transforms.keys():
            H, W = posed.img.shape[1:3]
            fov = stage_transforms[cls.HORIZONTAL_FOV_KEY]
            f = (W / 2) / math.tan(fov / 2)
            posed.intrinsics = np.array([[f, 0, W / 2 - 0.5], [0, f, H / 2 - 0.5], [0, 0, 1]])
        else:
            posed.intrinsics = np.array(stage_transforms[cls.INTRINSICS_KEY])
        return posed

    def transform_img(self, posed_imgs, alpha_over_white_bg, stage_transforms, renderer_params, camera_calibration):
        """:549-676 -> img (N, [3,] H, W) in the default dtype, normalised."""
        img = posed_imgs.img
        is_quantized = np.issubdtype(img.dtype, np.unsignedinteger)
        is_synthetic = renderer_params is not None
        num_img_channels = 1 if img.ndim == 3 else img.shape[3]
        bayer_pattern = str(camera_calibration[self.BAYER_PATTERN_KEY])
        if is_quantized:
            if self.BIT_DEPTH_KEY in stage_transforms.keys():
                levels = 2 ** stage_transforms[self.BIT_DEPTH_KEY]
            else:
                levels = int(np.iinfo(img.dtype).max) + 1
        interm = str(renderer_params[self.INTERM_COLOR_SPACE_KEY]) if is_synthetic else None
        _require(np.issubdtype(img.dtype, np.unsignedinteger) or np.issubdtype(img.dtype, np.floating),
                 f"images must be unsigned integers or floats, got {img.dtype}")
        _require(np.all(img >= 0), "negative pixel values")
        if is_synthetic:
            _require(interm == ("display" if is_quantized else "linear"),
                     f"{'quantised' if is_quantized else 'float'} renders with interm_color_space {interm!r}")
        else:
            _require(is_quantized, "real captures must be quantised")
        _require(num_img_channels in self.ACCEPTED_NUM_IMG_CHANNELS, f"{num_img_channels} image channels")
        if num_img_channels == 4:
            _require(is_synthetic, "only synthetic renders may carry an alpha channel")

        # alpha over a white background in the output colour space (:607-625)
        if alpha_over_white_bg:
            if interm == "display":  # straight alpha, f64 (an integer array over an int)
                alpha = (img[..., 3] / (levels - 1))[..., np.newaxis]
                img = alpha * img[..., :3] + (1 - alpha) * (levels - 1)
            elif interm == "linear":  # premultiplied alpha, f32
                alpha = img[..., 3][..., np.newaxis]
                img = img[..., :3] + (1 - alpha)
            else:  # the reference's own code has no branch for this (real captures, :610-623)
                raise AssertionError("alpha_over_white_bg needs synthetic renders (renderer_params.npz)")
        elif num_img_channels == 4:
            img = img[..., :3]
        img = img.astype(np.float32)

        if bayer_pattern != self.NULL_BAYER_PATTERN:  # (N, 3, H, W) RGB (:630-637)
            img = np.stack([image_io.bgr_to_rgb(x) for x in img], axis=0).transpose(0, 3, 1, 2)
        elif num_img_channels == 3:  # grey (:639-644)
            img = image_io.bgr_to_gray(img)

        # half-level normalisation of quantised values, else + log_eps (:646-670)
        if is_quantized:
            self.min_normalized_pixel_value = 0.5 / levels
            img = img / levels + self.min_normalized_pixel_value
            self.max_normalized_pixel_value = 1 - self.min_normalized_pixel_value
        else:
            self.min_normalized_pixel_value = float(renderer_params[self.LOG_EPS_KEY])
            img = img + np.float32(self.min_normalized_pixel_value)
            self.max_normalized_pixel_value = float(img.max())
        posed_imgs.img = torch.tensor(np.ascontiguousarray(img), dtype=torch.get_default_dtype())
        return posed_imgs

    @classmethod
    def transform_pose(cls, posed_imgs):
        """:678-702: the OpenGL camera frame (x right, y up, z back) to the common one (x right, y down,
        z forward) by a right multiplication; tensors in the default dtype (exposure_time as given)."""
        posed_imgs.T_wc_orientation = posed_imgs.T_wc_orientation @ cls.T_COPENGL_CCOMMON_ORIENTATION
        for k in ("T_wc_position", "T_wc_orientation", "intrinsics"):
            posed_imgs[k] = torch.tensor(posed_imgs[k], dtype=torch.get_default_dtype())
        if "gain" in posed_imgs.keys():
            posed_imgs.gain = torch.tensor(posed_imgs.gain, dtype=torch.get_default_dtype())
        if "exposure_time" in posed_imgs.keys():
            posed_imgs.exposure_time = torch.tensor(posed_imgs.exposure_time)
        return posed_imgs

    def __getitem__(self, index):
        return {k: v[index] for k, v in self.posed_imgs.items() if k != "intrinsics"}

    def __len__(self):
        return len(self.posed_imgs.img)


class CameraPose(torch.utils.data.Dataset):
    CAMERA_POSES_FILENAME = "camera_poses.npz"
    CAMERA_POSES_KEYS = {"T_wc_position", "T_wc_orientation", "T_wc_timestamp"}

    def __init__(self, root_directory, permutation_seed=None):
        super().__init__()
        self.camera_poses = self.load_camera_poses(root_directory)
        if permutation_seed is None:
            return
        g = torch.Generator()
        g.manual_seed(permutation_seed)
        perm = torch.randperm(len(self.camera_poses.T_wc_position), generator=g)
        for k, v in self.camera_poses.items():
            self.camera_poses[k] = v[perm]

    @classmethod
    def load_camera_poses(cls, root_directory):
        poses = EasyDict(dict(np.load(os.path.join(root_directory, cls.CAMERA_POSES_FILENAME), allow_pickle=False)))
        assert set(poses.keys()) == cls.CAMERA_POSES_KEYS
        for k, v in poses.items():
            poses[k] = torch.tensor(v)
        return poses

    @classmethod
    def from_arrays(cls, T_wc_position, T_wc_orientation, T_wc_timestamp):
        """A CameraPose from in-memory arrays (synthetic scenes, tests)."""
        obj = cls.__new__(cls)
        torch.utils.data.Dataset.__init__(obj)
        obj.camera_poses = EasyDict(T_wc_position=torch.as_tensor(T_wc_position),
                                    T_wc_orientation=torch.as_tensor(T_wc_orientation),
                                    T_wc_timestamp=torch.as_tensor(T_wc_timestamp))
        return obj

    def __getitem__(self, index):
        return {k: v[index] for k, v in self.camera_poses.items()}

    def __len__(self):
        return len(self.camera_poses.T_wc_position)
