"""On-disk formats: DRSA run selection and U loading, CNN checkpoints (CPU)."""
import os
import pickle

import numpy as np
import pandas as pd
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
