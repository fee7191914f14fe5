"""conv_onet decoder modules, API-compatible with src/conv_onet/models/decoder.py.

Parameter names, shapes, registration order and initialisers match the
reference, so ``state_dict``s (e.g. pretrained/middle_fine.pt) load unchanged and
a given ``torch.manual_seed`` yields the same weights:

  GaussianFourierFeatureTransform  decoder.py:7-30   (_B = randn(3,93)*25, learnable)
  DenseLayer                       decoder.py:70-85  (xavier_uniform(gain(act)), zero bias)
  MLP                              decoder.py:97-219 (fc_c[5], embedder, pts_linears[5], output_linear)
  MLP_no_xyz                       decoder.py:222-297
  NICE                             decoder.py:300-370

The modules only hold parameters.  Evaluation (``NICE.forward``) runs on the HIP
point-evaluation kernels of ``libnicecore.so`` (nicecore.ops.eval_points); there
is no PyTorch fallback on the product path.
"""
from __future__ import annotations

import torch
import torch.nn as nn

MAPPING_SIZE = 93
FOURIER_SCALE = 25


class GaussianFourierFeatureTransform(nn.Module):
    """sin(p @ B), B = randn(dim, 93) * 25 (decoder.py:17-30)."""

    def __init__(self, num_input_channels, mapping_size=MAPPING_SIZE, scale=FOURIER_SCALE,
                 learnable=True):
        super().__init__()
        B = torch.randn((num_input_channels, mapping_size)) * scale
        if learnable:
            self._B = nn.Parameter(B)
        else:
            self._B = B


class DenseLayer(nn.Linear):
    """nn.Linear with xavier-uniform init scaled by the activation gain (decoder.py:70-85)."""

    def __init__(self, in_dim: int, out_dim: int, activation: str = "relu", *args, **kwargs):
        self.activation = activation
        super().__init__(in_dim, out_dim, *args, **kwargs)

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain(self.activation))
        if self.bias is not None:
            nn.init.zeros_(self.bias)


class MLP(nn.Module):
    """Point decoder with xyz Fourier input and per-block feature injection.

    Only the configuration every NICE config uses is supported by the kernels:
    hidden 32, 5 blocks, skip after block 2, ``pos_embedding_method='fourier'``
    (configs/nice_slam.yaml:136); c_dim 32 (64 when ``concat_feature``).
    """

    def __init__(self, name='', dim=3, c_dim=128, hidden_size=256, n_blocks=5, leaky=False,
                 sample_mode='bilinear', color=False, skips=(2,), grid_len=0.16,
                 pos_embedding_method='fourier', concat_feature=False):
        super().__init__()
        if pos_embedding_method != 'fourier':
            raise NotImplementedError(
                "nicecore supports pos_embedding_method='fourier' only "
                "(the method every NICE config uses)")
        self.name = name
        self.color = color
        self.no_grad_feature = False
        self.c_dim = c_dim
        self.grid_len = grid_len
        self.concat_feature = concat_feature
        self.n_blocks = n_blocks
        self.skips = list(skips)
        self.hidden_size = hidden_size
        if c_dim != 0:
            self.fc_c = nn.ModuleList([nn.Linear(c_dim, hidden_size) for _ in range(n_blocks)])
        emb = MAPPING_SIZE
        self.embedder = GaussianFourierFeatureTransform(dim, mapping_size=emb, scale=FOURIER_SCALE)
        layers = [DenseLayer(emb, hidden_size, activation="relu")]
        for i in range(n_blocks - 1):
            fan_in = hidden_size + emb if i in self.skips else hidden_size
            layers.append(DenseLayer(fan_in, hidden_size, activation="relu"))
        self.pts_linears = nn.ModuleList(layers)
        self.output_linear = DenseLayer(hidden_size, 4 if color else 1, activation="linear")
        self.sample_mode = sample_mode
        self.leaky = leaky

    def forward(self, p, c_grid=None):
        """MLP.forward (decoder.py:190-219) for the iMAP* scene MLP (c_dim = 0, hidden 256,
        4 blocks, no skip: get_model(nice=False)) on the HIP kernels (nicecore.imap).  The
        NICE sub-decoders are evaluated together through NICE.forward."""
        if self.c_dim != 0:
            raise NotImplementedError("NICE sub-decoders are evaluated through NICE.forward(p, c_grid, stage)")
        from .imap import eval_points
        raw = eval_points(self, p)
        return raw if self.color else raw[:, 3]


class MLP_no_xyz(nn.Module):
    """Coarse decoder: grid feature only, skip concat of the feature after block 2
    (decoder.py:222-297)."""

    def __init__(self, name='', dim=3, c_dim=128, hidden_size=256, n_blocks=5, leaky=False,
                 sample_mode='bilinear', color=False, skips=(2,), grid_len=0.16):
        super().__init__()
        self.name = name
        self.no_grad_feature = False
        self.color = color
        self.grid_len = grid_len
        self.c_dim = c_dim
        self.n_blocks = n_blocks
        self.skips = list(skips)
        self.hidden_size = hidden_size
        layers = [DenseLayer(hidden_size, hidden_size, activation="relu")]
        for i in range(n_blocks - 1):
            fan_in = hidden_size + c_dim if i in self.skips else hidden_size
            layers.append(DenseLayer(fan_in, hidden_size, activation="relu"))
        self.pts_linears = nn.ModuleList(layers)
        self.output_linear = DenseLayer(hidden_size, 4 if color else 1, activation="linear")
        self.sample_mode = sample_mode
        self.leaky = leaky


class NICE(nn.Module):
    """Neural Implicit Scalable Encoding: coarse / middle / fine / color decoders
    (decoder.py:300-334).  ``forward(p, c_grid, stage)`` returns raw [P,4] with the
    reference's stage semantics (decoder.py:336-370), evaluated by the HIP kernels."""

    def __init__(self, dim=3, c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.16,
                 fine_grid_len=0.16, color_grid_len=0.16, hidden_size=32, coarse=False,
                 pos_embedding_method='fourier'):
        super().__init__()
        if c_dim != 32 or hidden_size != 32:
            raise NotImplementedError("nicecore kernels are built for c_dim=32, hidden_size=32")
        if coarse:
            self.coarse_decoder = MLP_no_xyz(name='coarse', dim=dim, c_dim=c_dim, color=False,
                                             hidden_size=hidden_size, grid_len=coarse_grid_len)
        self.middle_decoder = MLP(name='middle', dim=dim, c_dim=c_dim, color=False, skips=[2],
                                  n_blocks=5, hidden_size=hidden_size, grid_len=middle_grid_len,
                                  pos_embedding_method=pos_embedding_method)
        self.fine_decoder = MLP(name='fine', dim=dim, c_dim=c_dim * 2, color=False, skips=[2],
                                n_blocks=5, hidden_size=hidden_size, grid_len=fine_grid_len,
                                concat_feature=True, pos_embedding_method=pos_embedding_method)
        self.color_decoder = MLP(name='color', dim=dim, c_dim=c_dim, color=True, skips=[2],
                                 n_blocks=5, hidden_size=hidden_size, grid_len=color_grid_len,
                                 pos_embedding_method=pos_embedding_method)

    def forward(self, p, c_grid, stage='middle', **kwargs):
        from .ops import eval_points
        return eval_points(self, p, c_grid, stage)


def get_model(cfg, nice=True):
    """Factory with the signature of src/conv_onet/config.py:4-33."""
    if not nice:  # iMAP*: one scene MLP (config.py:28-32)
        return MLP(dim=cfg['data']['dim'], c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4,
                   pos_embedding_method=cfg['model']['pos_embedding_method'])
    return NICE(dim=cfg['data']['dim'], c_dim=cfg['model']['c_dim'], coarse=cfg['coarse'],
                coarse_grid_len=cfg['grid_len']['coarse'],
                middle_grid_len=cfg['grid_len']['middle'],
                fine_grid_len=cfg['grid_len']['fine'],
                color_grid_len=cfg['grid_len']['color'],
                pos_embedding_method=cfg['model']['pos_embedding_method'])


def build_default_nice(seed: int | None = 0, coarse: bool = True) -> NICE:
    """NICE with the configs/nice_slam.yaml hyper-parameters, seeded like the
    reference's ``get_model`` under ``torch.manual_seed(seed)``."""
    if seed is not None:
        torch.manual_seed(seed)
    return NICE(dim=3, c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.32,
                fine_grid_len=0.16, color_grid_len=0.16, hidden_size=32, coarse=coarse,
                pos_embedding_method='fourier')


def build_imap(seed: int | None = 0) -> MLP:
    """The iMAP* scene MLP of get_model(cfg, nice=False), seeded like the reference under
    ``torch.manual_seed(seed)``."""
    if seed is not None:
        torch.manual_seed(seed)
    return MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4,
               pos_embedding_method='fourier')
