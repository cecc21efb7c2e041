"""Concurrent batches on two HIP streams of one context (bench.py's launch form
for the fused-grid shapes, `--streams`): each stream's launches write their own
outputs, and every batch's outputs equal a single-stream launch of the same
frames bit for bit.  Only shapes whose launch keeps no per-context scratch
(Localizer.batch_grid_fused(), no least squares) are launched this way."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402


@pytest.mark.parametrize("engine", ["gcc_phat", "direct"])
def test_two_streams_equal_one(engine):
    loc = Localizer(engine=engine)
    assert loc.batch_grid_fused()
    lut = loc.lut().reshape(3, 101, 101)
    batches = [synth.adc_frames(4096, 3, 1024, lut, 46, 0x5151 + i, device="cuda")[0].contiguous()
               for i in range(6)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    outs = [[loc.alloc_outputs(4096) for _ in range(3)] for _ in range(2)]
    torch.cuda.synchronize()
    for rep in range(3):  # the same launches several times over: no state carried between them
        for i, fr in enumerate(batches):
            loc.prepare(fr, outs[i % 2][i // 2], streams[i % 2])()
    torch.cuda.synchronize()
    for i, fr in enumerate(batches):
        got = {k: v.cpu().numpy() for k, v in outs[i % 2][i // 2].items()}
        exp = {k: v.cpu().numpy() for k, v in loc.localize(fr).items()}
        for k in exp:
            assert np.array_equal(got[k], exp[k]), (engine, i, k)
    loc.close()
