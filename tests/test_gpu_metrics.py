"""GPU tests of the accuracy-metrics step (include/petmetrics.h, metrics.py) against
the reference's own NumPy calls (main_script.py:721-744: np.mean, np.cov, np.corrcoef)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('dtype,n,d', [(torch.float32, 10000, 96), (torch.float64, 777, 48), (torch.float64, 2, 5)])
def test_sample_moments_vs_numpy(dtype, n, d):
    from pet_posterior_distribution_amd.metrics import sample_moments
    rng = np.random.default_rng(n)
    x = (rng.standard_normal((n, d)) * rng.uniform(0.1, 3, d) + rng.uniform(-2, 2, d)).astype(
        np.float32 if dtype == torch.float32 else np.float64)
    mean, cov = sample_moments(torch.as_tensor(x, device='cuda'))
    np.testing.assert_allclose(mean.cpu().numpy(), x.astype(np.float64).mean(0), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(cov.cpu().numpy(), np.cov(x.astype(np.float64), rowvar=False), rtol=1e-9, atol=1e-12)


def test_posterior_metrics_match_reference_numpy():
    from pet_posterior_distribution_amd.metrics import posterior_metrics
    rng = np.random.default_rng(7)
    nn = rng.standard_normal((4000, 48, 2)).astype(np.float32) * 0.1 + 1.0
    mc = rng.standard_normal((3, 1500, 96)) * 0.1 + 1.2
    out = posterior_metrics(torch.as_tensor(nn, device='cuda'), torch.as_tensor(mc, device='cuda'))
    for p, name in enumerate(('DVR', 'R1')):
        a = mc[..., p * 48:(p + 1) * 48].reshape(-1, 48)
        b = nn[..., p].astype(np.float64)
        cov_a, cov_b = np.cov(a, rowvar=False), np.cov(b, rowvar=False)
        np.testing.assert_allclose(out[name]['cov']['MCMC'], cov_a, rtol=1e-9)
        np.testing.assert_allclose(out[name]['cov']['NN'], cov_b, rtol=1e-9, atol=1e-14)
        np.testing.assert_allclose(out[name]['corr']['NN'], np.corrcoef(b, rowvar=False) - np.eye(48), atol=1e-10)
        np.testing.assert_allclose(out[name]['mu']['Norm_diff'][:, 0],
                                   np.abs((a.mean(0) - b.mean(0)) / a.mean(0)), rtol=1e-8)
        np.testing.assert_allclose(out[name]['std']['NN'][:, 0], np.sqrt(np.diag(cov_b)), rtol=1e-9)
