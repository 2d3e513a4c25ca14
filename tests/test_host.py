"""Host-side logic on CPU: drop-in surface (src/ alias, main.py flags), U-Net
parameter init / state_dict parity with the reference layout, arena packing,
no silent CPU fallback, EarlyStopping and the metrics CSV."""
import csv

import pytest
import torch

from oracle import reference_torch as rt


def test_src_alias_imports_without_opencv():
    import src
    from src.loss import DiceBCEPDELoss
    from src.pde import PDERegularization, create_pde_regularization
    from src.train import EarlyStopping, train, train_stage, validate
    from src.unet import UNet
    import physics_informed_image_segmentation_amd as pkg
    assert src.UNet is pkg.UNet and UNet is pkg.UNet and DiceBCEPDELoss is pkg.DiceBCEPDELoss
    assert callable(train) and callable(train_stage) and callable(validate)
    assert isinstance(create_pde_regularization(5.0, 0.5), PDERegularization)


def test_unet_init_matches_reference_weights_and_keys():
    from physics_informed_image_segmentation_amd import UNet, count_parameters
    torch.manual_seed(42)
    net = UNet(1, 1, 64)
    torch.manual_seed(42)
    ref = rt.UNetRef(1, 1, 64)
    sd, rsd = net.state_dict(), ref.state_dict()
    assert list(sd) == list(rsd)
    for k in sd:
        assert sd[k].shape == rsd[k].shape and torch.equal(sd[k], rsd[k]), k
    assert count_parameters(net) == 20_543_809


def test_arena_views_and_layouts():
    from physics_informed_image_segmentation_amd import UNet
    net = UNet()
    base = net.arena.data_ptr()
    end = base + 4 * net.arena.numel()
    for p in net.parameters():
        assert base <= p.data_ptr() < end and (p.data_ptr() - base) % 256 == 0
    w = net.enc2.conv[0].weight  # (128, 64, 3, 3) stored KRSC
    assert w.stride() == (576, 1, 192, 64)
    wt = net.up4.weight  # (512, 512, 2, 2) stored [i][j][o][c]
    assert wt.stride() == (1, 512, 2 * 512 * 512, 512 * 512)
    # load_state_dict writes through the views into the arena
    ref = rt.UNetRef()
    net.load_state_dict(ref.state_dict())
    assert torch.equal(net.enc2.conv[0].weight, ref.enc2.conv[0].weight)
    assert net.enc2.conv[0].weight.data_ptr() >= base


def test_dtype_cast_refused_and_float_is_noop():
    from physics_informed_image_segmentation_amd import UNet
    net = UNet()
    ptrs = [p.data_ptr() for p in net.parameters()]
    net.float()
    assert [p.data_ptr() for p in net.parameters()] == ptrs
    with pytest.raises(NotImplementedError):
        net.double()


def test_no_cpu_fallback():
    from physics_informed_image_segmentation_amd import DiceBCEPDELoss, UNet
    from physics_informed_image_segmentation_amd._hip import HipError
    net = UNet()
    with pytest.raises(HipError):
        net(torch.zeros(1, 1, 32, 32))
    with pytest.raises(HipError):
        DiceBCEPDELoss()(torch.full((1, 1, 8, 8), 0.5), torch.zeros(1, 1, 8, 8))


def test_unsupported_configs_are_loud():
    from physics_informed_image_segmentation_amd import UNet
    with pytest.raises(ValueError):
        UNet(output_activation="softmax")
    with pytest.raises(NotImplementedError):
        UNet(output_activation="tanh")
    with pytest.raises(NotImplementedError):
        UNet(intermediate_activation="gelu")


def test_pde_constructor_checks_match_reference():
    from physics_informed_image_segmentation_amd import PDERegularization
    with pytest.raises(ValueError, match="diffusion_coeff must be positive"):
        PDERegularization(0.0)
    with pytest.raises(ValueError, match=r"reaction_threshold must be in \(0,1\)"):
        PDERegularization(1.0, 1.0)
    pr = PDERegularization(5.0, 0.5)
    assert pr.laplacian_kernel.shape == (1, 1, 3, 3)
    assert torch.equal(pr.grad_y_kernel[0, 0], torch.tensor([[0.0, -0.5, 0.0], [0.0, 0.0, 0.0], [0.0, 0.5, 0.0]]))
    with pytest.raises(ValueError, match="epsilon must be positive"):
        pr.compute_phase_field_loss(torch.zeros(1, 1, 4, 4), epsilon=0.0)


def test_loss_defaults_match_reference():
    from physics_informed_image_segmentation_amd import DiceBCELoss, DiceBCEPDELoss
    a = DiceBCELoss()
    assert (a.dice_weight, a.bce_weight, a.smooth) == (0.5, 0.5, 1e-6)
    b = DiceBCEPDELoss()
    assert (b.pde_weight, b.phase_field_weight, b.epsilon) == (1e-3, 0.0, 0.05)
    assert b.pde_regularization.diffusion_coeff == 1.0 and b.pde_regularization.reaction_threshold == 0.5


def test_early_stopping_semantics():
    from physics_informed_image_segmentation_amd import EarlyStopping
    es = EarlyStopping(patience=2, min_delta=1e-4, mode="max")
    assert not es(0.5, 1)
    assert not es(0.50005, 2)  # below min_delta: counter 1
    assert not es(0.6, 3)       # improvement resets
    assert not es(0.6, 4)
    assert es(0.6, 5)
    assert es.best_epoch == 3 and es.best_score == 0.6
    mn = EarlyStopping(patience=1, mode="min")
    mn(1.0, 1)
    assert mn(1.0, 2)


def test_metrics_csv_columns(tmp_path):
    from physics_informed_image_segmentation_amd.train import CSV_FIELDS, save_metrics_to_csv
    assert len(CSV_FIELDS) == 17
    rows = [{k: i for k in CSV_FIELDS} for i in range(3)]
    p = tmp_path / "out" / "m.csv"
    save_metrics_to_csv(rows, p)
    got = list(csv.DictReader(open(p)))
    assert list(got[0]) == CSV_FIELDS and len(got) == 3


def test_main_flags_and_defaults():
    import main
    a = main.parse_args([])
    assert (a.pde_weight, a.diffusion_coeff, a.reaction_threshold, a.phase_field_weight, a.epsilon) == \
        (1e-4, 5.0, 0.5, 1e-4, 0.05)
    assert (a.batch_size, a.learning_rate, a.stage1_epochs, a.stage2_epochs) == (8, 1e-4, 50, 50)
    assert a.early_stopping_patience == 5 and a.seed == 42 and not a.single_stage
    b = main.parse_args(["--single-stage", "--synthetic", "8", "4", "64", "64"])
    assert b.single_stage and b.synthetic == [8, 4, 64, 64]


def test_synthetic_dataset_deterministic():
    from physics_informed_image_segmentation_amd import SyntheticDiscDataset
    ds = SyntheticDiscDataset(4, (32, 48), seed=3)
    x1, m1 = ds[2]
    x2, m2 = ds[2]
    assert torch.equal(x1, x2) and torch.equal(m1, m2)
    assert x1.shape == (1, 32, 48) and set(m1.unique().tolist()) <= {0.0, 1.0}
    assert 0.0 <= x1.min() and x1.max() <= 1.0


def test_checkpoint_roundtrip_with_reference_layout(tmp_path):
    """.pth files are interchangeable with the reference's
    (src/train.py:688-690,763-764 torch.save(state_dict); src/evaluate_comparison.py:61-76
    load_state_dict(torch.load(...))), loadable with weights_only=True."""
    from physics_informed_image_segmentation_amd import UNet
    torch.manual_seed(3)
    net = UNet(1, 1, 64)
    torch.save(net.state_dict(), tmp_path / "ours.pth")
    sd = torch.load(tmp_path / "ours.pth", weights_only=True)
    ref = rt.UNetRef(1, 1, 64)
    ref.load_state_dict(sd)
    for (k, a), (k2, b) in zip(net.state_dict().items(), ref.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    torch.manual_seed(11)
    ref2 = rt.UNetRef(1, 1, 64)
    torch.save(ref2.state_dict(), tmp_path / "ref.pth")
    net.load_state_dict(torch.load(tmp_path / "ref.pth", weights_only=True))
    for (k, a), (_, b) in zip(net.state_dict().items(), ref2.state_dict().items()):
        assert torch.equal(a, b), k
    assert (tmp_path / "ours.pth").stat().st_size < 1.05 * (tmp_path / "ref.pth").stat().st_size
