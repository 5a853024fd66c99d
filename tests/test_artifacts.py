"""On-disk formats: DRSA run selection and U loading, CNN checkpoints (CPU)."""
import os
import pickle

import numpy as np
import pandas as pd
import pytest
import torch


def test_best_run_and_projection_matrix(tmp_path):
    from drsa_audio_amd.utils.evaluation import get_best_run, load_projection_matrix
    root = os.path.join(tmp_path, "blues", "layer7")
    for r, final in ((1, 0.3), (2, 0.5), (3, 0.4)):
        d = os.path.join(root, f"run{r}")
        os.makedirs(d)
        pd.DataFrame({"loss": np.linspace(0.1, final, 5).astype(np.float32)}).to_csv(os.path.join(d, "train_stats.csv"))
        with open(os.path.join(d, "projection_matrix.pkl"), "wb") as fh:
            pickle.dump(np.eye(4, dtype=np.float32) * r, fh)
    run, loss, _, path, losses = get_best_run(root)
    assert run == 2 and abs(loss - 0.5) < 1e-6 and path.endswith("run2") and len(losses) == 5
    U = load_projection_matrix("blues", 7, str(tmp_path))
    assert torch.equal(U, torch.eye(4) * 2)


def test_checkpoint_roundtrip_weights_only(tmp_path):
    from drsa_audio_amd.model.create_model import VGGType
    from drsa_audio_amd.utils.evaluation import load_checkpoint_state, save_checkpoint
    torch.manual_seed(0)
    m = VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5,
                input_size=(64, 64), conv_bn=True, dense_bn=True)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    p = save_checkpoint(str(tmp_path), m.state_dict(), opt.state_dict(), 1700)
    assert os.path.basename(p) == "best_model_1700.pth"
    m2 = VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5,
                 input_size=(64, 64), conv_bn=True, dense_bn=True)
    m2.load_state_dict(load_checkpoint_state(p))
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /dev/null",))


def test_safe_pickle_admits_arrays_and_refuses_code(tmp_path):
    from drsa_audio_amd.utils import safe_pickle
    p = tmp_path / "ok.pkl"
    arr = np.arange(12, dtype=np.float32).reshape(3, 4)
    pairs = list(zip(arr, arr * 2))                                    # save_data's numpy format
    tens = list(zip(torch.from_numpy(arr), torch.from_numpy(arr * 3)))  # the reference's torch rows
    for obj in (arr, pairs, tens):
        with open(p, "wb") as fh:
            pickle.dump(obj, fh)
        with open(p, "rb") as fh:
            back = safe_pickle.load(fh)
        if obj is arr:
            assert np.array_equal(back, arr)
        else:
            assert all(np.array_equal(np.asarray(a), np.asarray(b)) for x, y in zip(obj, back) for a, b in zip(x, y))
    with open(p, "wb") as fh:
        pickle.dump(_Evil(), fh)
    with open(p, "rb") as fh:
        with pytest.raises(pickle.UnpicklingError):
            safe_pickle.load(fh)


def test_dataset_file_roundtrip_formats(tmp_path):
    """dataset_layer{L}.pkl written with numpy rows (save_data here) or torch rows (the reference's
    save_data) reads back through the restricted loader (normalisation needs the GPU; the raw
    rows are checked here)."""
    from drsa_audio_amd.utils import safe_pickle
    from drsa_audio_amd.xai.drsa.cluster.getdrsadata import save_data
    A = np.random.default_rng(0).standard_normal((10, 8)).astype(np.float32)
    C = np.random.default_rng(1).standard_normal((10, 8)).astype(np.float32)
    path = save_data(A, C, layer=7, sample_class="blues", output_path=str(tmp_path))
    with open(path, "rb") as fh:
        a, c = zip(*safe_pickle.load(fh))
    assert np.array_equal(np.array(a), A) and np.array_equal(np.array(c), C)
