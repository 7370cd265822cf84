"""DataModule -- mirror of the reference's data/datamodule.py (DataModule, :8-289), so that
scripts/run.py:38-45 constructs it unchanged (``den.data.datamodule.DataModule(seed, eval_target,
num_nodes, gpus, pixel_bandwidth, **config.data)``).

It feeds the HIP training step: per rank, a random stream of event batches (``Event`` from
``events.pt``, batch = the dynamic size ``DeblurENeRF.update_train_batch_size`` sets) and the
normalized samples of the supervision timestamps (diff length = Dirac at 1, start positions
uniform, subdiff length triangular with mode 0, pixel-bandwidth interval generators Dirac at 0.5),
drawn from a per-rank generator seeded ``torch.initial_seed() + rank`` (:87-91) so DDP ranks see
different batches.  Main-process loading only (``num_workers_per_node == 0``, :42): the batch size
changes between steps.

A ``pytorch_lightning.LightningDataModule`` when Lightning is importable; otherwise a plain object
with the same attributes and loaders (Lightning is absent from this image).  The evaluation
datasets are ``PosedImage`` views (data/datasets.py); a directory without a ``views/`` folder still
trains (``setup("fit")`` leaves ``val_dataset`` None, where the reference would fail), while
``setup("validate" | "test")`` raises.
"""
import torch
import torch.distributed as dist

from ..utils import datasets as dataset_utils
from ..utils.easydict import EasyDict
from . import datasets, samplers

try:
    import pytorch_lightning as _pl
    _Base = _pl.LightningDataModule
    _HAS_PL = True
except ImportError:  # pragma: no cover - the image has no pytorch_lightning
    _Base = object
    _HAS_PL = False


class DataModule(_Base):
    def __init__(self, seed, eval_target, num_nodes, gpus, pixel_bandwidth, dataset_directory, train_dataset_ratio,
                 val_dataset_ratio, test_dataset_ratio, train_dataset_perm_seed, eval_dataset_perm_seed,
                 alpha_over_white_bg, train_init_eff_batch_size, train_eff_ray_sample_batch_size, val_eff_batch_size,
                 test_eff_batch_size, num_workers_per_node):
        super().__init__()
        for r in (train_dataset_ratio, val_dataset_ratio, test_dataset_ratio):
            if not (isinstance(r, int) or (isinstance(r, float) and 0.0 < r <= 1.0)):
                raise ValueError(f"dataset ratio {r!r}: an int (batches) or a float in (0, 1]")
        if num_workers_per_node != 0:
            raise ValueError("num_workers_per_node must be 0: the training batch size changes between steps "
                             "(datamodule.py:37-42)")
        self.eval_target = eval_target
        self.pixel_bandwidth = pixel_bandwidth
        self.dataset_directory = dataset_directory
        self.train_dataset_ratio = train_dataset_ratio
        self.val_dataset_ratio = val_dataset_ratio
        self.test_dataset_ratio = test_dataset_ratio
        self.train_dataset_perm_seed = train_dataset_perm_seed
        self.eval_dataset_perm_seed = eval_dataset_perm_seed
        self.alpha_over_white_bg = alpha_over_white_bg
        self.val_eff_batch_size = val_eff_batch_size
        self.test_eff_batch_size = test_eff_batch_size
        hp = dict(seed=seed, train_init_eff_batch_size=train_init_eff_batch_size,
                  train_eff_ray_sample_batch_size=train_eff_ray_sample_batch_size)
        if _HAS_PL:
            self.save_hyperparameters(hp)
        else:
            self._hparams = EasyDict(hp)
        # per-GPU batch sizes (:64-80); gpus None = one CPU process
        n = 1 if gpus is None else num_nodes * len(gpus)
        self.train_batch_size = train_init_eff_batch_size // n
        self.val_batch_size = val_eff_batch_size // n
        self.test_batch_size = test_eff_batch_size // n
        self.num_workers = num_workers_per_node if gpus is None else num_workers_per_node // len(gpus)
        self.train_dataset = self.val_dataset = self.test_dataset = None
        self.train_normalized_sampler = None
        self.train_generator = None

    if not _HAS_PL:
        @property
        def hparams(self):
            return self._hparams

    # ------------------------------------------------------------------ setup
    def setup(self, stage=None):
        if stage in (None, "fit"):
            # distinct streams per DDP rank (:85-91)
            seed = torch.initial_seed()
            if dist.is_available() and dist.is_initialized():
                seed += dist.get_rank()
            self.train_generator = torch.Generator()
            self.train_generator.manual_seed(seed)
            self.train_dataset = self._build_dataset("train")
            self.val_dataset = self._build_eval_dataset("val", required=False)
            self.train_normalized_sampler = self._build_normalized_sampler()
        if stage in (None, "validate"):
            self.val_dataset = self._build_eval_dataset("val", required=True)
        if stage in (None, "test"):
            self.test_dataset = self._build_eval_dataset("test", required=True)

    def _subset(self, dataset, stage):
        ratio = {"train": self.train_dataset_ratio, "val": self.val_dataset_ratio,
                 "test": self.test_dataset_ratio}[stage]
        if isinstance(ratio, int):
            eff = {"train": self.hparams.train_init_eff_batch_size, "val": self.val_eff_batch_size,
                   "test": self.test_eff_batch_size}[stage]
            length = ratio * eff
            if length > len(dataset):
                raise ValueError(f"{stage}: {ratio} batches of {eff} exceed the {len(dataset)} items")
        else:
            length = int(ratio * len(dataset))
        return dataset_utils.TrimDataset(dataset, 0, length)

    def _build_dataset(self, stage):
        """The training events (:101-149): Event -> trimmed -> endless random batches."""
        assert stage == "train"
        ev = self._subset(datasets.Event(self.dataset_directory, self.train_dataset_perm_seed), "train")
        return dataset_utils.IterableMapDataset(ev, self.train_batch_size, self.train_generator)

    def _build_eval_dataset(self, stage, required):
        """The evaluation views (:107-119): PosedImage of the training views' images for an
        ``event_view`` target, else of the stage's own transforms; permuted by
        ``eval_dataset_perm_seed``, alpha-composited over white when configured, trimmed (:121-139)."""
        if datasets.PosedImage.posed_img_folder_path(self.dataset_directory) is None:
            if required:
                raise FileNotFoundError(f"no views/ folder in or above {self.dataset_directory} (PosedImage)")
            return None  # training-only directory: fit proceeds without a val set
        if set(self.eval_target) == {"event_view"}:
            ds = datasets.PosedImage(self.dataset_directory, "train", self.eval_dataset_perm_seed,
                                     self.alpha_over_white_bg)
        elif set(self.eval_target) == {"novel_view"}:
            ds = datasets.PosedImage(self.dataset_directory, stage, self.eval_dataset_perm_seed,
                                     self.alpha_over_white_bg)
        else:
            raise NotImplementedError(f"eval_target {self.eval_target}")
        return self._subset(ds, stage)

    def _build_normalized_sampler(self):
        """ts_diff / diff_start_ts / ts_subdiff / subdiff_start_ts (+ interval_gen) (:151-213)."""
        n, g, f64 = self.train_batch_size, self.train_generator, torch.float64
        parts = {"ts_diff": samplers.DiracDeltaSampler(1, n, f64),
                 "diff_start_ts": samplers.UniformSampler(0, 1, n, f64, g),
                 "ts_subdiff": samplers.TriangularSampler(0, 1, n, 0, f64, g),
                 "subdiff_start_ts": samplers.UniformSampler(0, 1, n, f64, g)}
        if self.pixel_bandwidth.enable:
            parts["interval_gen"] = samplers.DiracDeltaSampler(0.5, (self.pixel_bandwidth.it_sample_size - 1, n),
                                                               f64)
        return dataset_utils.JoinDataset(list(parts.values()), list(parts.keys()))

    # ------------------------------------------------------------------ loaders
    def _loader(self, dataset, batch_size):
        return torch.utils.data.DataLoader(dataset, batch_size=batch_size, num_workers=self.num_workers,
                                           shuffle=False, pin_memory=torch.cuda.is_available(), drop_last=False,
                                           persistent_workers=self.num_workers > 0)

    def train_dataloader(self):
        """{"event": batches of the dynamic size, "normalized": the matching samples} (:215-247);
        batch_size 1 adds the leading dim training_step squeezes."""
        return {"event": self._loader(self.train_dataset, 1),
                "normalized": self._loader(self.train_normalized_sampler, 1)}

    def val_dataloader(self):
        return self._loader(self.val_dataset, self.val_batch_size)

    def test_dataloader(self):
        return self._loader(self.test_dataset, self.test_batch_size)
