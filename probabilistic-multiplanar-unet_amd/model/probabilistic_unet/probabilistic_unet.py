"""Probabilistic U-Net — drop-in for PMU/model/probabilistic_unet/probabilistic_unet.py (rows a9-a12).

Same constructors, attributes, module tree (hence state_dict keys) and RNG consumption as the
reference, so seeded construction and checkpoints are interchangeable.  The compute runs on the
HIP path:
  * Encoder + latent head  -> one autograd node per AxisAlignedConvGaussian (pmu_hip.functions.
    GaussianFunction): conv3x3/BN/ReLU with AvgPool2d(2,ceil) fused into operand staging, spatial
    mean and the 1x1 latent conv as HIP kernels.
  * Fcomb                  -> one node (FcombFunction): fused per-pixel MLP on MFMA, z folded in
    as a per-sample bias instead of tiling it over H x W.
  * UNet features          -> model.UNet(apply_last_layer=False) on the HIP path.
The distributions (Independent(Normal)) and the analytic KL on (N, latent_dim) tensors are the same
torch.distributions the reference uses; the summed cross entropy runs on pmu_hip.loss.
"""
import torch
import torch.nn as nn
from torch.distributions import Independent, Normal, kl

from ..unet import UNet
from .utils import init_weights, init_weights_orthogonal_normal, l2_regularisation  # noqa: F401

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")   # module global, as in :9


def _fns():
    from pmu_hip import functions
    return functions


class Encoder(nn.Module):
    """len(num_filters) blocks of [AvgPool2d(2,2,ceil) except first] + no_convs_per_block x
    (Conv3x3 -> BatchNorm2d -> ReLU) (probabilistic_unet.py:11-53)."""

    def __init__(self, input_channels, num_filters, no_convs_per_block, initializers, padding=True, posterior=False):
        super().__init__()
        self.contracting_path = nn.ModuleList()
        self.input_channels = input_channels + (1 if posterior else 0)   # the concatenated mask (:22-24)
        self.num_filters = num_filters
        layers = []
        cin = self.input_channels
        for i, cout in enumerate(num_filters):
            if i != 0:
                layers.append(nn.AvgPool2d(kernel_size=2, stride=2, padding=0, ceil_mode=True))
            for j in range(no_convs_per_block):
                layers.append(nn.Conv2d(cin if j == 0 else cout, cout, kernel_size=3, padding=int(padding)))
                layers.append(nn.BatchNorm2d(cout))
                layers.append(nn.ReLU(inplace=True))
            cin = cout
        self.layers = nn.Sequential(*layers)
        self.layers.apply(init_weights)

    def forward(self, input):
        """The encoding (N, num_filters[-1], h, w).  AxisAlignedConvGaussian.forward does not call this:
        it runs encoder + mean + latent head as one fused node; a direct call is its own node."""
        return _fns().encoder_apply(self, input)


class AxisAlignedConvGaussian(nn.Module):
    """Encoder -> spatial mean -> 1x1 conv to (mu, log_sigma) -> Independent(Normal) (:55-114)."""

    def __init__(self, input_channels, num_filters, no_convs_per_block, latent_dim, initializers, posterior=False):
        super().__init__()
        self.input_channels = input_channels
        self.channel_axis = 1
        self.num_filters = num_filters
        self.no_convs_per_block = no_convs_per_block
        self.latent_dim = latent_dim
        self.posterior = posterior
        self.name = "Posterior" if posterior else "Prior"
        self.encoder = Encoder(self.input_channels, self.num_filters, self.no_convs_per_block, initializers,
                               posterior=self.posterior)
        self.conv_layer = nn.Conv2d(num_filters[-1], 2 * self.latent_dim, (1, 1), stride=1)
        self.show_img = 0
        self.show_seg = 0
        nn.init.kaiming_normal_(self.conv_layer.weight, mode="fan_in", nonlinearity="relu")
        nn.init.normal_(self.conv_layer.bias)

    # the reference's debug attributes (:85-93), computed when read instead of on every forward
    @property
    def show_concat(self):
        """cat(input, segm) of the last forward that had a mask (0 before any)."""
        if not isinstance(self.show_seg, torch.Tensor):
            return 0
        return torch.cat((self.show_img, self.show_seg), dim=1)

    @property
    def sum_input(self):
        c = self.show_concat
        return torch.sum(c) if isinstance(c, torch.Tensor) else 0

    @property
    def show_enc(self):
        """The encoder output of the last forward (relu(bn) of its last conv, NCHW-shaped)."""
        return _fns().gaussian_encoding(self)

    def forward(self, input, segm=None):
        if segm is not None:
            self.show_img = input
            self.show_seg = segm
        mu_log_sigma = _fns().gaussian_apply(self, input, segm)
        mu = mu_log_sigma[:, :self.latent_dim]
        log_sigma = mu_log_sigma[:, self.latent_dim:]
        return Independent(Normal(loc=mu, scale=torch.exp(log_sigma)), 1)


class Fcomb(nn.Module):
    """no_convs_fcomb 1x1 convs on cat(features, tile(z)) (:116-181)."""

    def __init__(self, num_filters, latent_dim, num_output_channels, num_classes, no_convs_fcomb, initializers,
                 use_tile=True):
        super().__init__()
        self.num_channels = num_output_channels
        self.num_classes = num_classes
        self.channel_axis = 1
        self.spatial_axes = [2, 3]
        self.num_filters = num_filters
        self.latent_dim = latent_dim
        self.use_tile = use_tile
        self.no_convs_fcomb = no_convs_fcomb
        self.name = "Fcomb"
        if self.use_tile:
            f0 = self.num_filters[0]
            layers = [nn.Conv2d(f0 + self.latent_dim, f0, kernel_size=1), nn.ReLU(inplace=True)]
            for _ in range(no_convs_fcomb - 2):
                layers += [nn.Conv2d(f0, f0, kernel_size=1), nn.ReLU(inplace=True)]
            self.layers = nn.Sequential(*layers)
            self.last_layer = nn.Conv2d(f0, self.num_classes, kernel_size=1)
            init = init_weights_orthogonal_normal if initializers["w"] == "orthogonal" else init_weights
            self.layers.apply(init)
            self.last_layer.apply(init)

    def tile(self, a, dim, n_tile):
        """tf.tile semantics along ``dim`` (:155-165); kept for API parity — forward never tiles."""
        idx = torch.arange(a.size(dim), device=a.device).repeat_interleave(n_tile)
        return torch.index_select(a, dim, idx)

    def forward(self, feature_map, z):
        if self.use_tile:
            return _fns().fcomb_apply(self, feature_map, z)
        return None

    def forward_samples(self, feature_map, zs):
        """S latent samples in one pass over the features: zs (S,N,L) -> (S,N,K,H,W) (no autograd)."""
        return _fns().fcomb_samples(self, feature_map, zs)


class ProbabilisticUnet(nn.Module):
    """A probabilistic U-Net (https://arxiv.org/abs/1806.05034), :184-308."""

    def __init__(self, input_channels=1, num_classes=1, num_filters=[32, 64, 128, 192], latent_dim=6,
                 no_convs_fcomb=3, beta=1.0):
        super().__init__()
        self.n_channels = input_channels
        self.n_classes = num_classes
        self.num_filters = num_filters
        self.latent_dim = latent_dim
        self.no_convs_per_block = 2
        self.no_convs_fcomb = no_convs_fcomb
        self.initializers = {"w": "he_normal", "b": "normal"}
        self.beta = beta
        self.z_prior_sample = 0
        self.unet = UNet(n_channels=self.n_channels, n_classes=self.n_classes, num_filters=self.num_filters,
                         apply_last_layer=False).to(device)
        self.prior = AxisAlignedConvGaussian(self.n_channels, self.num_filters, self.no_convs_per_block,
                                             self.latent_dim, self.initializers).to(device)
        self.posterior = AxisAlignedConvGaussian(self.n_channels, self.num_filters, self.no_convs_per_block,
                                                 self.latent_dim, self.initializers, posterior=True).to(device)
        self.fcomb = Fcomb(self.num_filters, self.latent_dim, self.n_channels, self.n_classes, self.no_convs_fcomb,
                           {"w": "orthogonal", "b": "normal"}, use_tile=True).to(device)
        fns = _fns()
        for sub in (self.unet, self.prior, self.posterior, self.fcomb):
            fns.set_grad_root(sub, self)   # one flat gradient buffer for the whole model
        self.posterior_latent_space = None
        self.prior_latent_space = None
        self.unet_features = None

    def forward(self, patch, segm, training=True):
        """Prior latent space and UNet features for ``patch``; the posterior too when training (:215-223).
        The three parts are independent: on the HIP path they run on concurrent streams
        (pmu_hip.functions.run_concurrent; PMU_PROB_STREAMS=0 runs them in the reference's order)."""
        from pmu_hip.engine import CFG
        if CFG.prob_streams and isinstance(patch, torch.Tensor) and patch.is_cuda:
            parts = [lambda: self.unet.forward(patch), lambda: self.prior.forward(patch)]
            if training:
                parts.append(lambda: self.posterior.forward(patch, segm))
            res = _fns().run_concurrent(patch.device, parts)
            self.unet_features, self.prior_latent_space = res[0], res[1]
            if training:
                self.posterior_latent_space = res[2]
            return
        if training:
            self.posterior_latent_space = self.posterior.forward(patch, segm)
        self.prior_latent_space = self.prior.forward(patch)
        self.unet_features = self.unet.forward(patch)

    def sample(self, testing=False):
        """Segmentation logits from a prior sample (rsample when training, sample when testing) (:225-240)."""
        if testing is False:
            z_prior = self.prior_latent_space.rsample()
        else:
            z_prior = self.prior_latent_space.sample()
        self.z_prior_sample = z_prior
        return self.fcomb.forward(self.unet_features, z_prior)

    def sample_many(self, n, testing=True):
        """``n`` prior samples through Fcomb in one fused pass: (n, N, K, H, W).  Extension of
        sample() for the evaluation sweep (visualize_sampling / GED); draws like ``sample``."""
        d = self.prior_latent_space
        zs = d.sample((n,)) if testing else d.rsample((n,)).detach()
        return self.fcomb.forward_samples(self.unet_features, zs)

    def sample_at(self, z):
        """Logits at latent location ``z``.  z (L,): batch-1 features, as in the reference (:242-247),
        -> (1, K, H, W).  Extension: z (S, L), S locations (e.g. latent_grid's) decoded in one fused
        pass over the features (read once) -> (S, N, K, H, W), for features of any batch N."""
        z = z.to(device=self.unet_features.device, dtype=torch.float32)
        if z.dim() == 1:
            return self.fcomb.forward(self.unet_features, z.unsqueeze(0))
        N = self.unet_features.shape[0]
        return self.fcomb.forward_samples(self.unet_features, z[:, None, :].expand(z.shape[0], N, z.shape[1]))

    @staticmethod
    def latent_grid(n_preds, mu, sigma, dims=(0, 1)):
        """The latent sweep of visualize_sampling.visualize_sample (visualize_sampling.py:22-26):
        z[dims[0]] = mu + a*sigma, z[dims[1]] = mu + b*sigma for a, b in range(-(n//2), n//2 + 1), the
        other components at mu.  Returns (rows*cols, L), row-major (a outer)."""
        mu, sigma = mu.reshape(-1).float(), sigma.reshape(-1).float()
        ks = torch.arange(-(n_preds // 2), n_preds // 2 + 1, dtype=torch.float32, device=mu.device)
        a, b = torch.meshgrid(ks, ks, indexing="ij")
        z = mu.repeat(a.numel(), 1)
        z[:, dims[0]] = a.reshape(-1) * sigma[dims[0]] + mu[dims[0]]
        z[:, dims[1]] = b.reshape(-1) * sigma[dims[1]] + mu[dims[1]]
        return z

    def reconstruct(self, use_posterior_mean=False, calculate_posterior=False, z_posterior=None):
        """Decode a posterior sample (or its mean) with the UNet features (:251-262)."""
        if use_posterior_mean:
            z_posterior = self.posterior_latent_space.loc
        elif calculate_posterior:
            z_posterior = self.posterior_latent_space.rsample()
        return self.fcomb.forward(self.unet_features, z_posterior)

    def kl_divergence(self, analytic=True, calculate_posterior=False, z_posterior=None):
        """KL(Q||P) per image, analytic or by a posterior sample (:264-279)."""
        if analytic:
            return kl.kl_divergence(self.posterior_latent_space, self.prior_latent_space)
        if calculate_posterior:
            z_posterior = self.posterior_latent_space.rsample()
        return self.posterior_latent_space.log_prob(z_posterior) - self.prior_latent_space.log_prob(z_posterior)

    def elbo(self, segm, analytic_kl=True, reconstruct_posterior_mean=False):
        """-(sum CE(reconstruction, segm) + beta * mean KL) (:281-308)."""
        if self.n_classes == 1:
            criterion = nn.BCEWithLogitsLoss(reduction="none")
        else:
            from pmu_hip.loss import CrossEntropyLoss   # HIP kernels; the sum of :304 fused in
            criterion = CrossEntropyLoss(reduction="sum")
        z_posterior = self.posterior_latent_space.rsample()
        self.kl = torch.mean(self.kl_divergence(analytic=analytic_kl, calculate_posterior=False,
                                                z_posterior=z_posterior))
        self.reconstruction = self.reconstruct(use_posterior_mean=reconstruct_posterior_mean,
                                               calculate_posterior=False, z_posterior=z_posterior)
        self.reconstruction = self.reconstruction.to(device=device, dtype=torch.float32)
        segm = segm.to(device=device, dtype=torch.long).squeeze(1)
        reconstruction_loss = criterion(input=self.reconstruction, target=segm)
        self.reconstruction_loss = torch.sum(reconstruction_loss)
        return -(self.reconstruction_loss + self.beta * self.kl)
