"""Dataset adaptors of the training data path -- the reference's utils/datasets.py (:5-49).

* ``JoinDataset``: zips several endless iterable datasets into dicts keyed by name (the
  normalized-sample loader of DataModule, datamodule.py:151-164).
* ``IterableMapDataset``: turns a map-style dataset into an endless stream of random batches
  drawn with replacement, ``batch_size`` read anew for every batch so that
  ``DeblurENeRF.update_train_batch_size`` can resize it between steps (:20-32).
* ``TrimDataset``: the first ``end - start`` items of a dataset (indexing is passed through
  unchanged, as the reference does: :35-49).

Host-side plumbing: the batches are index gathers on CPU tensors, copied to the device by the
loader (pin_memory) before ``training_step`` runs.
"""
import torch


class JoinDataset(torch.utils.data.IterableDataset):
    def __init__(self, datasets, dataset_keys):
        datasets, dataset_keys = list(datasets), list(dataset_keys)
        if not all(isinstance(d, torch.utils.data.IterableDataset) for d in datasets):
            raise TypeError("JoinDataset joins iterable-style datasets")
        if not all(isinstance(k, str) for k in dataset_keys):
            raise TypeError("JoinDataset keys are strings")
        self.datasets = datasets
        self.dataset_keys = dataset_keys

    def __iter__(self):
        streams = [iter(d) for d in self.datasets]
        while True:
            item = {}
            for key, stream in zip(self.dataset_keys, streams):
                try:
                    item[key] = next(stream)
                except StopIteration:
                    return
            yield item


class IterableMapDataset(torch.utils.data.IterableDataset):
    def __init__(self, map_dataset, batch_size, generator=None):
        self.map_dataset = map_dataset
        self.batch_size = batch_size
        self.generator = generator

    def __iter__(self):
        n = len(self.map_dataset)
        while True:
            idx = torch.randint(n, (self.batch_size,), generator=self.generator)
            yield self.map_dataset[idx]


class TrimDataset(torch.utils.data.Dataset):
    def __init__(self, dataset, start_index, end_index):
        if end_index < start_index:
            raise ValueError("TrimDataset: end_index < start_index")
        self.dataset = dataset
        self.start_index = start_index
        self.trimmed_len = end_index - start_index

    def __len__(self):
        return self.trimmed_len

    def __getitem__(self, index):
        return self.dataset[index]
