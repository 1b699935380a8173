"""Multi-planar MRI slice dataset — drop-in for PMU/utils/mri_dataset.py:11-143 (row a13).

Same constructor (imgs_dir, masks_dir, n_classes, filter=True), attributes (ids, views,
image_dims, index_map, len) and item format ({'image': (1,H,W) f32, 'mask': (1,H,W) f32}), and
the same semantics:
  * pad_dimensions: zeros appended to the end of the argmin axis up to the max dim (:85-98);
  * index map ordered scan -> view -> slice, keeping slices whose mask max > 0 when ``filter``
    (:37-49); views are image[i,:,:], image[:,j,:], image[:,:,k] (:70-82);
  * preprocess: image / its own max when that max is non-zero, mask untouched (:101-112).

MI355X-first differences:
  * every scan is read from disk ONCE and kept resident in HBM (the reference re-reads the
    whole volume from disk for every slice, :124-127), re-laid out per view so that each slice
    is one contiguous block (pmu_slice_view_layout, f64 so that the max normalisation is
    bit-identical to the reference's numpy arithmetic);
  * the index-map filter and the normalisation maxima come from one per-slice max reduction per
    view (pmu_slice_max);
  * items are produced on the GPU; ``get_batch(indices)`` assembles a whole batch in one launch
    per tensor (pmu_gather_slices) — what the training loop uses instead of a DataLoader.

``loader`` (path -> ndarray) defaults to nibabel's ``nib.load(path).get_fdata()``; nibabel is an
optional dependency.  ``files`` replaces ``listdir(imgs_dir)`` (the reference's, unsorted order).
"""
from __future__ import annotations

import logging
from os import listdir, path

import numpy as np
import torch
from torch.utils.data import Dataset
from torch.utils.data.dataloader import default_collate

from pmu_hip import _lib as L


def _nib_load(p):
    try:
        import nibabel as nib
    except ImportError as e:  # pragma: no cover - depends on the host
        raise ImportError("MRI_Dataset needs nibabel to read NIfTI scans (or pass loader=...)") from e
    return nib.load(p).get_fdata()


def padded_shape(shape):
    """pad_dimensions' output shape: the (first) argmin axis grows by max - min (:85-98)."""
    shape = list(shape)
    diff = max(shape) - min(shape)
    if diff:
        shape[int(np.argmin(shape))] += diff
    return tuple(shape)


def view_slice_shape(pshape, view):
    p0, p1, p2 = pshape
    return [(p1, p2), (p0, p2), (p0, p1)][view]


class _ScanViews:
    """One scan resident in HBM: per-view contiguous layouts of image and mask, per-slice maxima."""

    def __init__(self, img: np.ndarray, mask: np.ndarray, device):
        if img.ndim != 3 or mask.ndim != 3:
            raise ValueError("MRI_Dataset expects 3-D scans")
        self.pshape = padded_shape(img.shape)
        if padded_shape(mask.shape) != self.pshape:
            raise AssertionError(f"Image and mask should be the same size, but are {img.shape} and {mask.shape}")
        s = L.stream()
        self.img, self.mask, self.img_max, self.mask_max = [], [], [], []
        for vol, views, maxes in ((img, self.img, self.img_max), (mask, self.mask, self.mask_max)):
            d = torch.from_numpy(np.ascontiguousarray(vol, dtype=np.float64)).to(device)
            d0, d1, d2 = vol.shape
            p0, p1, p2 = self.pshape
            for v in range(3):
                out = torch.empty(p0 * p1 * p2, dtype=torch.float64, device=device)
                L.call("pmu_slice_view_layout", d.data_ptr(), d0, d1, d2, p0, p1, p2, v, out.data_ptr(), s)
                n = self.pshape[v]
                ha, hb = view_slice_shape(self.pshape, v)
                mx = torch.empty(n, dtype=torch.float64, device=device)
                L.call("pmu_slice_max", out.data_ptr(), n, ha * hb, mx.data_ptr(), s)
                views.append(out)
                maxes.append(mx)
            del d


class MRI_Dataset(Dataset):

    def __init__(self, imgs_dir, masks_dir, n_classes, filter=True, loader=None, files=None, device=None):
        self.imgs_dir = imgs_dir
        self.masks_dir = masks_dir
        self.n_classes = n_classes
        self.len = 0
        self.views = self.initialize_views(use_standard_axis=True)
        self.ids = list(files) if files is not None else listdir(imgs_dir)
        self._load = loader or _nib_load
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise RuntimeError("MRI_Dataset keeps scans resident on the GPU (there is no CPU fallback)")
        logging.info("Creating index mapping.")
        self.scans = []
        self.image_dims = None
        self.index_map = []
        for scan, name in enumerate(self.ids):
            img = self._load(path.join(self.imgs_dir, name))
            mask = self._load(path.join(self.masks_dir, name))
            if self.image_dims is None:   # largest dim of the first scan, per axis (:28-29)
                self.image_dims = tuple([int(np.max(img.shape))] * len(img.shape))
            sv = _ScanViews(np.asarray(img), np.asarray(mask), self.device)
            self.scans.append(sv)
            fg = [(m > 0).cpu().numpy() for m in sv.mask_max]
            for view in range(len(self.views)):
                for sl in range(sv.pshape[view]):
                    if not filter or fg[view][sl]:
                        self.index_map.append((scan, view, sl))
        self.len = len(self.index_map)
        self._build_table()
        logging.info(f"Creating dataset of {len(self.ids)} scans, and {self.len} slices")

    def _build_table(self):
        """Device slice table for pmu_gather_slices: address and max of every (scan, view, slice)."""
        addr_i, addr_m, max_i, self._gid, self._shape = [], [], [], {}, {}
        for scan, sv in enumerate(self.scans):
            for v in range(3):
                ha, hb = view_slice_shape(sv.pshape, v)
                px = ha * hb
                for sl in range(sv.pshape[v]):
                    self._gid[(scan, v, sl)] = len(addr_i)
                    self._shape[(scan, v, sl)] = (ha, hb)
                    addr_i.append(sv.img[v].data_ptr() + sl * px * 8)
                    addr_m.append(sv.mask[v].data_ptr() + sl * px * 8)
            max_i.extend(sv.img_max)
        self._addr_img = torch.tensor(addr_i, dtype=torch.int64).to(self.device)
        self._addr_mask = torch.tensor(addr_m, dtype=torch.int64).to(self.device)
        self._max_img = torch.cat(max_i) if max_i else torch.empty(0, dtype=torch.float64, device=self.device)

    def __len__(self):
        return self.len

    def initialize_views(self, use_standard_axis=False):
        """Standard axes (:60-66)."""
        standard_axis = [np.array([1, 0, 0]), np.array([0, 1, 0]), np.array([0, 0, 1])]
        if use_standard_axis:
            return standard_axis
        raise ValueError("only the standard axes are defined (as in the reference)")

    def sample_slice(self, image, view, slice_index):
        """Host-side slice of an array (:70-82), kept for API parity."""
        if np.array_equal(view, self.views[0]):
            return image[slice_index, :, :]
        if np.array_equal(view, self.views[1]):
            return image[:, slice_index, :]
        if np.array_equal(view, self.views[2]):
            return image[:, :, slice_index]
        raise ValueError("No valid view")

    def pad_dimensions(self, image):
        """Host-side pad (:85-98), kept for API parity; the resident path pads on the GPU."""
        out = np.zeros(padded_shape(image.shape), dtype=image.dtype)
        out[:image.shape[0], :image.shape[1], :image.shape[2]] = image
        return out

    @classmethod
    def preprocess(cls, img, label=False):
        """(H,W) -> (1,H,W), image / max when max != 0 (:101-112) — host-side, for API parity."""
        if len(img.shape) == 2:
            img = np.expand_dims(img, axis=2)
        img_trans = np.transpose(img, [2, 0, 1])
        if not label and not np.max(img_trans) == 0:
            img_trans = img_trans / np.max(img_trans)
        return img_trans

    def get_batch(self, indices):
        """{'image': (B,1,H,W), 'mask': (B,1,H,W)} f32 on the GPU for dataset indices (one launch each)."""
        return self.get_slices([self.index_map[int(i)] for i in indices])

    def get_slices(self, keys):
        """Same as get_batch for explicit (scan, view, slice) keys (also slices the filter dropped)."""
        shapes = {self._shape[k] for k in keys}
        if len(shapes) != 1:
            raise RuntimeError(f"slices of one batch must share a shape, got {sorted(shapes)}")
        ha, hb = shapes.pop()
        B = len(keys)
        ids = torch.tensor([self._gid[k] for k in keys], dtype=torch.int32).to(self.device, non_blocking=True)
        img = torch.empty(B, 1, ha, hb, dtype=torch.float32, device=self.device)
        mask = torch.empty(B, 1, ha, hb, dtype=torch.float32, device=self.device)
        s = L.stream()
        L.call("pmu_gather_slices", self._addr_img.data_ptr(), self._max_img.data_ptr(), ids.data_ptr(), B, ha * hb,
               1, img.data_ptr(), s)
        L.call("pmu_gather_slices", self._addr_mask.data_ptr(), None, ids.data_ptr(), B, ha * hb, 0,
               mask.data_ptr(), s)
        return {"image": img, "mask": mask}

    def __getitem__(self, i):
        b = self.get_batch([i])
        return {"image": b["image"][0], "mask": b["mask"][0]}


def mri_collate(batch):
    """Collate that drops None items (train.py imports it; the reference file does not define it)."""
    return default_collate([b for b in batch if b is not None])
