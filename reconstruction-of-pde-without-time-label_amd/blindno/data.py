"""Datasets of the reference's train scripts: file formats, physical scaling and
normalisation, item layout -- plus an HBM-resident view for the GPU trainer.

Reference Dataset classes (defined inside the flat train scripts):
  TrajectoryDataset2D       2d_FPE/train_fno.py:11-60  (npz keys trajectories, potential, drag;
                            scales 1e10 / 1e21 / 1e6; z-score: trajectories over axes (0, 1),
                            targets over axis 0; std + 1e-8; item y = (Nx, Ny, 2))
  TrajectoryDataset2DForce  2d_Non_conservative_FPE/train_fno.py:13-60 (the reference also names
                            it TrajectoryDataset2D; npz keys trajectories, F (M, 2, Nx, Ny);
                            F scale 1e12; item y = F.permute(1, 2, 0))
  TrajectoryDataset1D       1d_FPE/train_fno.py:8-58   (scales 1e5 / 1e20 / 1e5; drag (M,) is
                            a scalar repeated over x; item y = stack(potential, drag) (Nx, 2))
  ParameterDataset          1d_GPE/train_fno_GPE.py:33-74 (np.save'd dict y, g, kappa, V;
                            y and V divided by max/3, g and kappa by their max; item y = V[:, None])
The arithmetic is the reference's own numpy sequence (float32 arrays, same reductions, same
order), so the normalised arrays match bit for bit (tests/test_data.py against fixtures captured
from the reference classes).  Normalisation is host-side work in the reference and stays on the
host here; ``device_tensors`` moves a normalised split into HBM once for the trainer.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset


def _zscore(a: np.ndarray, axis) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    mean = a.mean(axis=axis, keepdims=True)
    std = a.std(axis=axis, keepdims=True) + 1e-8
    return (a - mean) / std, mean, std


class TrajectoryDataset2D(Dataset):
    """2D FPE bags (drift potential + drag targets), 2d_FPE/train_fno.py:11-60."""

    def __init__(self, file_path: Optional[str] = None, *, arrays: Optional[dict] = None):
        data = arrays if arrays is not None else np.load(file_path)   # npz: no pickles needed
        self.trajectories = np.array(data["trajectories"], dtype=np.float32) * 1e10
        self.potential = np.array(data["potential"], dtype=np.float32) * 1e21
        self.drag = np.array(data["drag"], dtype=np.float32) * 1e6
        self.trajectories, self.trajectories_mean, self.trajectories_std = _zscore(self.trajectories, (0, 1))
        self.potential, self.potential_mean, self.potential_std = _zscore(self.potential, 0)
        self.drag, self.drag_mean, self.drag_std = _zscore(self.drag, 0)

    def __len__(self):
        return len(self.trajectories)

    def __getitem__(self, idx):
        x = torch.tensor(self.trajectories[idx], dtype=torch.float32)
        y = torch.cat((torch.tensor(self.potential[idx], dtype=torch.float32).unsqueeze(-1),
                       torch.tensor(self.drag[idx], dtype=torch.float32).unsqueeze(-1)), axis=2)
        return x, y

    def targets(self) -> np.ndarray:
        return np.stack([self.potential, self.drag], axis=-1)


class TrajectoryDataset2DForce(Dataset):
    """2D non-conservative FPE bags (force Fx, Fy targets), 2d_Non_conservative_FPE/train_fno.py:13-60."""

    def __init__(self, file_path: Optional[str] = None, *, arrays: Optional[dict] = None):
        data = arrays if arrays is not None else np.load(file_path)
        self.trajectories = np.array(data["trajectories"], dtype=np.float32) * 1e10
        self.F = np.array(data["F"], dtype=np.float32) * 1e12
        self.trajectories, self.trajectories_mean, self.trajectories_std = _zscore(self.trajectories, (0, 1))
        self.F, self.F_mean, self.F_std = _zscore(self.F, 0)

    def __len__(self):
        return len(self.trajectories)

    def __getitem__(self, idx):
        x = torch.tensor(self.trajectories[idx], dtype=torch.float32)
        y = torch.tensor(self.F[idx], dtype=torch.float32).permute(1, 2, 0)
        return x, y

    def targets(self) -> np.ndarray:
        return np.ascontiguousarray(np.transpose(self.F, (0, 2, 3, 1)))


class TrajectoryDataset1D(Dataset):
    """1D FPE bags (potential + scalar drag), 1d_FPE/train_fno.py:8-58."""

    def __init__(self, file_path: Optional[str] = None, *, arrays: Optional[dict] = None):
        data = arrays if arrays is not None else np.load(file_path)
        self.trajectories = np.array(data["trajectories"], dtype=np.float32) * 1e5
        self.potential = np.array(data["potential"], dtype=np.float32) * 1e20
        self.drag = np.array(data["drag"], dtype=np.float32) * 1e5
        self.drag = self.drag[:, np.newaxis]
        self.trajectories, self.trajectories_mean, self.trajectories_std = _zscore(self.trajectories, (0, 1))
        self.potential, self.potential_mean, self.potential_std = _zscore(self.potential, 0)
        self.drag, self.drag_mean, self.drag_std = _zscore(self.drag, 0)

    def __len__(self):
        return len(self.trajectories)

    def __getitem__(self, idx):
        x = torch.tensor(self.trajectories[idx], dtype=torch.float32)
        pot = torch.tensor(self.potential[idx], dtype=torch.float32)
        drag = torch.tensor(self.drag[idx], dtype=torch.float32).repeat(pot.shape[0])
        return x, np.stack((pot, drag), axis=1)

    def targets(self) -> np.ndarray:
        return np.stack([self.potential, np.repeat(self.drag, self.potential.shape[1], 1)], -1)


_NUMPY_PICKLE_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
}


def load_npy_dict(path: str) -> dict:
    """A dict of arrays / numbers saved with ``np.save(path, dict)`` (the GPE generator's
    format, 1d_GPE/datagen_GPE.py:183-189), read WITHOUT ``allow_pickle``: the object payload
    is unpickled by a restricted unpickler that resolves only numpy's array / dtype / scalar
    reconstructors -- any other global in the file (code execution) raises."""
    import pickle

    class _Restricted(pickle.Unpickler):
        def find_class(self, module, name):
            if (module, name) in _NUMPY_PICKLE_GLOBALS:
                return super().find_class(module, name)
            raise pickle.UnpicklingError(f"{path}: refusing to load global {module}.{name}")

    with open(path, "rb") as f:
        version = np.lib.format.read_magic(f)
        if version == (1, 0):
            shape, _, dtype = np.lib.format.read_array_header_1_0(f)
        else:
            shape, _, dtype = np.lib.format.read_array_header_2_0(f)
        if dtype != np.dtype(object):
            raise ValueError(f"{path}: not an np.save'd object (dict) file")
        arr = _Restricted(f).load()
    obj = arr.item() if isinstance(arr, np.ndarray) else arr
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: payload is {type(obj).__name__}, expected dict")
    return obj


class ParameterDataset(Dataset):
    """1D GPE bags (potential V target), 1d_GPE/train_fno_GPE.py:33-74.  ``file_path`` is the
    generator's np.save'd dict (1d_GPE/datagen_GPE.py:183-189), read with ``load_npy_dict``
    (restricted unpickler: numpy arrays and scalars only)."""

    def __init__(self, file_path: Optional[str] = None, *, arrays: Optional[dict] = None,
                 verbose: bool = False):
        data = arrays if arrays is not None else load_npy_dict(file_path)
        self.y = data["y"]
        self.g = data["g"]
        self.kappa = data["kappa"]
        self.V = data["V"]
        self.y_max = self.y.max() / 3
        self.V_max = self.V.max() / 3
        self.g_max = self.g.max()
        self.kappa_max = self.kappa.max()
        if verbose:
            print("Scaling factors:")
            print("y_max:", self.y_max, "V_max:", self.V_max, "g_max:", self.g_max,
                  "kappa_max:", self.kappa_max)
        self.y = self.y / self.y_max
        self.V = self.V / self.V_max
        self.g = self.g / self.g_max
        self.kappa = self.kappa / self.kappa_max

    def __len__(self):
        return len(self.y)

    def __getitem__(self, idx):
        target = np.stack([self.V[idx]], axis=-1)
        return torch.tensor(self.y[idx], dtype=torch.float32), torch.tensor(target, dtype=torch.float32)

    def targets(self) -> np.ndarray:
        return self.V[..., None].astype(np.float32)


def device_tensors(ds, indices: Optional[Sequence[int]] = None, device="cuda"):
    """(X, Y) of the (optionally subset) dataset as contiguous fp32 tensors in HBM, in the
    item layout the models consume: X (n, T, *grid), Y (n, *grid, C).  One host->device copy;
    the trainer then gathers batches on the device."""
    x = ds.trajectories if hasattr(ds, "trajectories") else ds.y
    y = ds.targets()
    if indices is not None:
        idx = np.asarray(indices)
        x, y = x[idx], y[idx]
    X = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(device)
    Y = torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).to(device)
    return X, Y
