"""Dataset file formats / normalisation against fixtures captured from
the reference's own Dataset classes (tests/golden/make_golden_data.py).  Host-side, CPU."""
import numpy as np
import torch

from conftest import load_golden


def _items(ds):
    xs, ys = zip(*[ds[i] for i in range(len(ds))])
    return torch.stack(xs).numpy(), np.stack([np.asarray(y) for y in ys])


def test_trajectory_dataset_2d_fpe():
    from blindno.data import TrajectoryDataset2D, device_tensors
    g = load_golden("dataset_2d_fpe")
    ds = TrajectoryDataset2D(arrays={k: g[k] for k in ("trajectories", "potential", "drag")})
    x, y = _items(ds)
    assert np.array_equal(x, g["x"]) and np.array_equal(y, g["y"])
    for a, b in (("trajectories_mean", "traj_mean"), ("trajectories_std", "traj_std"),
                 ("potential_mean", "pot_mean"), ("drag_std", "drag_std")):
        assert np.array_equal(getattr(ds, a), g[b])
    X, Y = device_tensors(ds, device="cpu")
    assert np.array_equal(X.numpy(), g["x"]) and np.array_equal(Y.numpy(), g["y"])


def test_trajectory_dataset_2d_force():
    from blindno.data import TrajectoryDataset2DForce, device_tensors
    g = load_golden("dataset_2d_nc")
    ds = TrajectoryDataset2DForce(arrays={"trajectories": g["trajectories"], "F": g["F"]})
    x, y = _items(ds)
    assert np.array_equal(x, g["x"]) and np.array_equal(y, g["y"])
    assert np.array_equal(ds.F_mean, g["F_mean"]) and np.array_equal(ds.F_std, g["F_std"])
    X, Y = device_tensors(ds, indices=[3, 1], device="cpu")
    assert np.array_equal(Y.numpy(), g["y"][[3, 1]])


def test_trajectory_dataset_1d():
    from blindno.data import TrajectoryDataset1D, device_tensors
    g = load_golden("dataset_1d_fpe")
    ds = TrajectoryDataset1D(arrays={k: g[k] for k in ("trajectories", "potential", "drag")})
    x, y = _items(ds)
    assert np.array_equal(x, g["x"]) and np.array_equal(y, g["y"])
    X, Y = device_tensors(ds, device="cpu")
    assert np.array_equal(Y.numpy(), g["y"])


def test_parameter_dataset_gpe(tmp_path):
    from blindno.data import ParameterDataset
    from blindno.gpe import save_training_data
    g = load_golden("dataset_1d_gpe")
    d = {"y": g["y_raw"], "g": g["g"], "kappa": g["kappa"], "V": g["V_raw"]}
    save_training_data(d, str(tmp_path / "d.npy"))               # the reference's file format
    ds = ParameterDataset(str(tmp_path / "d.npy"))
    x, t = _items(ds)
    assert np.array_equal(x, g["x"]) and np.array_equal(t, g["t"])
    assert ds.y_max == g["y_max"] and ds.V_max == g["V_max"]


def test_load_npy_dict_restricted(tmp_path):
    """The GPE generator's np.save'd dict reads back through the restricted unpickler (arrays
    and numpy scalars), and a file carrying any other global is refused."""
    import pickle
    import numpy as np
    import pytest
    from blindno.data import load_npy_dict
    d = {"y": np.random.rand(3, 5, 8), "g": np.float64(2.0), "kappa": np.arange(3.0), "V": np.ones((3, 8))}
    np.save(tmp_path / "ok.npy", d, allow_pickle=True)
    got = load_npy_dict(str(tmp_path / "ok.npy"))
    assert sorted(got) == sorted(d) and all(np.array_equal(got[k], d[k]) for k in d)

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))
    arr = np.empty((), dtype=object)
    arr[()] = {"y": Evil()}
    with open(tmp_path / "bad.npy", "wb") as f:
        np.lib.format.write_array_header_1_0(f, {"descr": "|O", "fortran_order": False, "shape": ()})
        pickle.dump(arr, f, protocol=3)
    with pytest.raises(pickle.UnpicklingError, match="refusing"):
        load_npy_dict(str(tmp_path / "bad.npy"))
