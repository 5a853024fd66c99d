"""Constants of the reference (``cxai/utils/constants.py``) built on this package's rules."""
from ..zennit.rules import Epsilon, Flat, Gamma, WSquare

CLASS_IDX_MAPPER = {"pop": 0, "metal": 1, "disco": 2, "blues": 3, "reggae": 4, "classical": 5, "rock": 6,
                    "hiphop": 7, "country": 8, "jazz": 9}
CLASS_IDX_MAPPER_TOY = {"class1": 0, "class2": 1}

AUDIO_PARAMS = {
    "gtzan": {"sample_rate": 16000, "slice_length": 3, "num_chunks": 8, "n_fft": 800, "hop_length": 360,
              "n_mels": 128, "mel_width": 128},
    "toy": {"sample_rate": 16000, "slice_length": 1, "num_chunks": 1, "n_fft": 480, "hop_length": 240,
            "n_mels": 64, "mel_width": 64},
}

# reference constants.py:27-38
LRP_NAME_MAP_GTZAN = [
    (["features.0"], WSquare(stabilizer=1e-7)),
    (["features.3"], Gamma(gamma=0.4, stabilizer=1e-7)),
    (["features.6"], Gamma(gamma=0.4, stabilizer=1e-7)),
    (["features.9"], Gamma(gamma=0.4 / 2, stabilizer=1e-7)),
    (["features.12"], Gamma(gamma=0.4 / 4, stabilizer=1e-7)),
    (["classifier.0"], Epsilon(epsilon=1e-7)),
    (["classifier.3"], Epsilon(epsilon=1e-7)),
    (["classifier.6"], Epsilon(epsilon=1e-7)),
]

# reference constants.py:40-51
LRP_NAME_MAP_TOY = [
    (["features.0"], Flat(stabilizer=1e-7)),
    (["features.3"], Gamma(gamma=0.8, stabilizer=1e-7)),
    (["features.6"], Gamma(gamma=0.8, stabilizer=1e-7)),
    (["features.9"], Gamma(gamma=0.8, stabilizer=1e-7)),
    (["features.12"], Gamma(gamma=0.8, stabilizer=1e-7)),
    (["classifier.0"], Epsilon(epsilon=1e-7)),
    (["classifier.2"], Epsilon(epsilon=1e-7)),
    (["classifier.4"], Epsilon(epsilon=1e-7)),
]


def lrp_name_map_vggish(gamma: float = 0.3, stab: float = 1e-7, dense_eps: float = 1e-7):
    """VGGish-BN name map of the reference's DRSA data script (getdrsadata.py:87-108): WSquare on
    the first conv, Gamma(gamma) on blocks 1-2, gamma/2 on blocks 3-4, gamma/4 on block 5,
    Epsilon on the dense layers (the model is used with SequentialMergeBatchNorm)."""
    return [
        (["features.0"], WSquare(stabilizer=stab)),
        (["features.3"], Gamma(gamma=gamma, stabilizer=stab)),
        (["features.7"], Gamma(gamma=gamma, stabilizer=stab)),
        (["features.10"], Gamma(gamma=gamma, stabilizer=stab)),
        (["features.14"], Gamma(gamma=gamma / 2, stabilizer=stab)),
        (["features.17"], Gamma(gamma=gamma / 2, stabilizer=stab)),
        (["features.21"], Gamma(gamma=gamma / 2, stabilizer=stab)),
        (["features.24"], Gamma(gamma=gamma / 2, stabilizer=stab)),
        (["features.28"], Gamma(gamma=gamma / 4, stabilizer=stab)),
        (["features.31"], Gamma(gamma=gamma / 4, stabilizer=stab)),
        (["classifier.0"], Epsilon(epsilon=dense_eps)),
        (["classifier.4"], Epsilon(epsilon=dense_eps)),
        (["classifier.8"], Epsilon(epsilon=dense_eps)),
    ]


LRP_NAME_MAP_VGGISH = lrp_name_map_vggish()
