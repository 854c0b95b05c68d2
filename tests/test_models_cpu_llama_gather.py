"""The vocab-parallel next-token all-gather that rides the xGMI SUM all-reduce
(models/llama.py gather_rows_for_sum / gathered_from_sum) is exact: every
rank's f32 (value, index) pairs -- infinities, denormals and large vocab
indices included -- come back bit-identical after an f32-accumulated sum of the
bf16 byte rows, rounded to bf16 as the kernel stores it."""
import torch

from ray_dynamic_batching_amd.models.llama import gather_rows_for_sum, gathered_from_sum


def test_byte_rows_sum_is_an_exact_gather():
    g = torch.Generator().manual_seed(0)
    for world, B in ((2, 1), (8, 4), (8, 13)):
        locs = [torch.stack([torch.randn(B, generator=g) * 50,
                             torch.randint(0, 128256, (B,), generator=g).float()], -1) for _ in range(world)]
        locs[world - 1][0, 0] = float("-inf")
        locs[0][-1, 0] = 1e-40                               # f32 denormal
        acc = None
        for r in range(world):
            buf = gather_rows_for_sum(locs[r], r, world, torch.bfloat16)
            assert buf.shape[1] % 8 == 0
            acc = buf.float() if acc is None else acc + buf.float()
        out = gathered_from_sum(acc.to(torch.bfloat16), locs[0])
        assert out.shape == (world, B, 2)
        for r in range(world):
            assert torch.equal(out[r].view(torch.int32), locs[r].view(torch.int32))


def test_byte_rows_reject_other_widths():
    import pytest

    with pytest.raises(ValueError):
        gather_rows_for_sum(torch.zeros(4, dtype=torch.float16), 0, 2, torch.bfloat16)
