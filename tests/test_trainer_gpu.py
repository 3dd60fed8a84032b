"""The trainer mirror driving the HIP generators with fused metrics (PSNR/SSIM
with denormalize inside the kernels) and HIP losses: the validation log
equals the reference loop's values computed with the oracle metrics on the
same outputs (1e-4 relative for PSNR/loss, 1e-4 absolute for SSIM), and a
few training epochs lower the loss."""
import pytest
import torch
from torch.utils.data import DataLoader

from oracle import cpu_nets
from vsr_amd import losses, metrics, nets
from vsr_amd.data import SyntheticCine
from vsr_amd.runner import trainers

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _run(trainer_cls, net, ds, vsr):
    loader = DataLoader(ds, batch_size=4, shuffle=False)
    tr = trainer_cls(device=DEV, train_dataloader=loader, valid_dataloader=loader, net=net,
                     loss_fns=[losses.L1Loss()], loss_weights=[1.0], metric_fns=[metrics.PSNR(), metrics.SSIM()],
                     optimizer=torch.optim.Adam(net.parameters(), lr=1e-3), lr_scheduler=None, logger=None,
                     monitor=None, num_epochs=1)
    got, _, _ = tr._run_epoch("validation")
    # the reference loop on the same outputs, oracle metrics on the CPU
    acc = {"Loss": 0.0, "L1Loss": 0.0, "PSNR": 0.0, "SSIM": 0.0}
    count = 0
    with torch.no_grad():
        for b in loader:
            if vsr:
                xs = [x.to(DEV) for x in b["lr_imgs"]]
                outs = [o.cpu() for o in net(xs)]
                ys = b["hr_imgs"]
                l1 = torch.stack([torch.nn.functional.l1_loss(o, y) for o, y in zip(outs, ys)]).mean().item()
                den = [(cpu_nets.denormalize(o, "acdc"), cpu_nets.denormalize(y, "acdc")) for o, y in zip(outs, ys)]
                ps = torch.stack([cpu_nets.psnr(o, y) for o, y in den]).mean().item()
                ss = torch.stack([cpu_nets.ssim(o, y) for o, y in den]).mean().item()
                w = loader.batch_size * len(xs)
            else:
                out = net(b["lr_img"].to(DEV)).cpu()
                y = b["hr_img"]
                l1 = torch.nn.functional.l1_loss(out, y).item()
                o_d, y_d = cpu_nets.denormalize(out, "acdc"), cpu_nets.denormalize(y, "acdc")
                ps, ss = cpu_nets.psnr(o_d, y_d).item(), cpu_nets.ssim(o_d, y_d).item()
                w = loader.batch_size
            for k, v in (("Loss", l1), ("L1Loss", l1), ("PSNR", ps), ("SSIM", ss)):
                acc[k] += v * w
            count += w
    ref = {k: v / count for k, v in acc.items()}
    assert list(got) == list(ref)
    for k in ("Loss", "L1Loss", "PSNR"):
        assert abs(got[k] - ref[k]) <= 1e-4 * abs(ref[k]), (k, got[k], ref[k])
    assert abs(got["SSIM"] - ref["SSIM"]) <= 1e-4, (got["SSIM"], ref["SSIM"])
    first = tr._run_epoch("training")[0]["Loss"]
    for _ in range(3):
        last = tr._run_epoch("training")[0]["Loss"]
    assert last < first


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_sisr_trainer_edsr(precision):
    torch.manual_seed(0)
    net = nets.EDSRNet(1, 1, num_resblocks=2, num_features=32, upscale_factor=2).to(DEV).set_precision(precision)
    _run(trainers.AcdcSISRTrainer, net, SyntheticCine("sisr", volumes=2, frames=4, size=(16, 24), upscale_factor=2),
         vsr=False)


def test_vsr_trainer_drf():
    torch.manual_seed(0)
    net = nets.DRFNet(1, 1, num_features=32, num_groups=2, upscale_factor=2).to(DEV).set_precision("fp32")
    _run(trainers.AcdcVSRTrainer, net, SyntheticCine("vsr", volumes=4, frames=3, size=(12, 16), upscale_factor=2),
         vsr=True)
