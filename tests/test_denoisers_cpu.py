"""CPU checks of the restated denoisers (no GPU needed): DRUNet layout / size / FLOPs, the
DenoiserPrior arithmetic order (sampling_images.py:156-157)."""
import torch

from psgla_for_posterior_sampling_amd.denoisers import (DenoiserPrior, DnCNN, DRUNet, dncnn_flops_per_pixel,
                                                        drunet_flops_per_pixel)


def test_drunet_layout_and_size():
    m = DRUNet()
    assert sum(p.numel() for p in m.parameters()) == 32640960      # KAIR / deepinv drunet_color
    keys = list(m.state_dict())
    assert keys[0] == "m_head.weight" and keys[-1] == "m_tail.weight"
    assert "m_down1.4.weight" in keys and "m_up3.0.weight" in keys and "m_body.3.res.2.weight" in keys
    assert abs(drunet_flops_per_pixel() * 256 * 256 / 1e9 - 277.55) < 0.1


def test_drunet_odd_sizes_and_sigma_map():
    torch.manual_seed(0)
    m = DRUNet(nc=(8, 16, 32, 64), nb=1)
    with torch.no_grad():
        for shape in [(1, 3, 24, 40), (2, 3, 24, 47), (1, 3, 100, 72), (1, 3, 16, 16)]:
            x = torch.rand(shape)
            assert m(x, 0.02).shape == x.shape
        x = torch.rand(1, 3, 16, 24)
        assert torch.equal(m(x, 0.02), m(x, torch.tensor([0.02])))


def test_dncnn_size():
    assert sum(p.numel() for p in DnCNN().parameters()) == 668227
    assert abs(dncnn_flops_per_pixel() * 65536 / 1e9 - 87.43) < 0.01


def test_denoiser_prior_matches_reference_closure():
    torch.manual_seed(1)
    den = DnCNN(depth=3, nf=8)
    s1 = 5 / 255.0
    alphat, s2t = torch.tensor(1.0), torch.tensor(s1 ** 2)
    x = torch.rand(1, 3, 16, 16)
    Ds = lambda x: den.forward(x, s1)                    # noqa: E731  (sampling_images.py:156-157)
    ref = lambda x: alphat * (Ds(x) - x) / s2t           # noqa: E731
    with torch.no_grad():
        assert torch.equal(DenoiserPrior(den, s1, alphat, s2t)(x), ref(x))


def test_drunet_size_dispatch_follows_deepinv():
    """deepinv 0.2.1 DRUNet.forward's routes (KAIR utils_model): forward_unet in eval mode for sides
    % 8 == 0 and > 31, test_pad(modulo 16) in training mode or when a side is < 32, test_onesplit(refield 64) otherwise.  With an
    elementwise stand-in for the U-Net every route returns exactly 2 x its input (the stitching is
    checked pixel for pixel); the recorded input shapes name the route."""
    m = DRUNet(nc=(8, 16, 32, 64), nb=1)
    seen = []

    def unet(x):
        seen.append(tuple(x.shape[-2:]))
        return 2 * x[:, :3]
    m.forward_unet = unet
    with torch.no_grad():
        for (h, w), shapes in [((64, 40), [(64, 40)]),                     # multiples of 8, > 31
                               ((24, 40), [(32, 48)]),                     # a side < 32: pad to 16
                               ((16, 16), [(16, 16)]),                     # < 32, already a multiple
                               ((481, 321), [(256, 192)] * 4),             # CBSD68 / castle: onesplit
                               ((321, 481), [(192, 256)] * 4),
                               ((100, 72), [(64, 64)] * 4)]:
            seen.clear()
            x = torch.rand(1, 3, h, w)
            y = m(x, 0.05)
            assert seen == shapes, (h, w, seen)
            assert torch.equal(y, 2 * x), (h, w)
        # training mode: test_pad(modulo 16) at every size (deepinv takes forward_unet only in eval mode)
        m.train()
        for (h, w), shape in [((64, 40), (64, 48)), ((100, 72), (112, 80)), ((64, 64), (64, 64))]:
            seen.clear()
            x = torch.rand(1, 3, h, w)
            y = m(x, 0.05)
            assert seen == [shape], (h, w, seen)
            assert torch.equal(y, 2 * x), (h, w)


def test_dncnn_backward_matches_pytorch_with_grad():
    """With autograd on, DnCNN runs the plain conv + bias + ReLU graph (the fused HIP epilogue is only
    taken without a gradient), so its backward is PyTorch's."""
    torch.manual_seed(2)
    den = DnCNN(depth=3, nf=8, channels_last=False)
    x = torch.rand(1, 3, 12, 12, requires_grad=True)
    den.forward(x).sum().backward()
    g = x.grad.clone()
    x.grad = None
    ref = torch.nn.functional.relu(den.in_conv(x))
    ref = torch.nn.functional.relu(den.conv_list[0](ref))
    (den.out_conv(ref) + x).sum().backward()
    assert torch.allclose(g, x.grad)
