"""BASELINE config 5 per rank: waveforms resident in HBM -> the reference sampler's batch layout
(K = 1024 classes x M = 2 clips, ContrastiveBatchSampler) -> 4096 MFCC / SpecAugment views built
on the GPU (GpuViewBuilder, the reference's per-(index, view) seeds) -> one cnn_deep bf16 train
step (forward, SupCon, backward, FusedAdam).  Properties at full size: view shape [2048, 2, 1,
40, 201], unit-norm embeddings, finite loss and gradients, and a bit-identical repeat (same
indices, same seeds, same dropout masks)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_config5_views_to_deep_bf16_step_b4096():
    from phoneme_contrast_amd.data import GpuContrastiveBatches, ShardedBatchSampler, WaveformStore
    from phoneme_contrast_amd.features import GpuViewBuilder, MFCCExtractor
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import model_registry
    from phoneme_contrast_amd.samplers import ContrastiveBatchSampler
    from phoneme_contrast_amd.transforms import FrequencyMask, GaussianNoise, TimeMask, Compose

    dev = torch.device("cuda")
    store = WaveformStore.synthetic(2048, 2, 32000, seed=7, device=dev)
    sampler = ContrastiveBatchSampler(store.labels, classes_per_batch=1024, samples_per_class=2, views_per_sample=2,
                                      seed=42)
    aug = Compose([TimeMask(30, 0.5), FrequencyMask(10, 0.5), GaussianNoise(0.001, 0.005, 0.3)])
    loader = GpuContrastiveBatches(store, ShardedBatchSampler(sampler, 0, 1),
                                   GpuViewBuilder(MFCCExtractor(), aug, 2, "train"))
    batch = next(iter(loader))
    views, labels = batch["views"], batch["label"]
    assert tuple(views.shape) == (2048, 2, 1, 40, 201) and torch.isfinite(views).all()
    x = views.reshape(4096, 1, 40, 201)
    y = labels.to(dev).repeat_interleave(2)
    # each class appears M * V = 4 times, consecutively (the trainer's flatten of the sampler layout)
    assert (y.view(-1, 4) == y.view(-1, 4)[:, :1]).all()

    torch.manual_seed(42)
    model = model_registry.create("phoneme_cnn_deep", {"embedding_dim": 128, "use_attention": True,
                                                       "dropout_rate": 0.2, "precision": "bf16"}).to(dev).train()
    loss_fn = SupervisedContrastiveLoss(temperature=0.15)
    res = []
    for _ in range(2):
        torch.manual_seed(123)  # same Dropout2d masks
        for p in model.parameters():
            p.grad = None
        e = model(x)
        loss = loss_fn(e, y)
        loss.backward()
        res.append((e.detach().clone(), loss.item(), torch.cat([p.grad.reshape(-1) for p in model.parameters()])))
    e, loss, g = res[0]
    assert torch.allclose(e.norm(dim=1), torch.ones(4096, device=dev), atol=1e-5)
    assert np.isfinite(loss) and torch.isfinite(g).all() and g.abs().max() > 0
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1] and torch.equal(res[0][2], res[1][2])
    # the batch is rebuilt identically from the same indices
    b2 = next(iter(GpuContrastiveBatches(store, [next(iter(ShardedBatchSampler(
        ContrastiveBatchSampler(store.labels, 1024, 2, 2, seed=42), 0, 1)))],
        GpuViewBuilder(MFCCExtractor(), aug, 2, "train"))))
    assert torch.equal(b2["views"], views)
