"""SCAFFOLD aggregation on the GPU vs the reference's own ``scaffold_aggregate_fn`` outputs
(scaffold.py:149-189; tests/golden/scaffold_cases.*, make_golden.py --set scaffold).

Params and control differences are summed by the HIP engine in one helper (controls under a reserved key
prefix, split back afterwards): bit-exact params and controls (NaN payloads excepted), the reference's key
order, containers and dtypes, metrics and meta exactly equal.  The controls add no launches of their own."""

import pytest

from golden_util import check_scaffold_result, load_scaffold_golden, scaffold_models_from_case
from nvflare_amd.app_common.workflows import aggregate_fn
from nvflare_amd.app_common.workflows.scaffold import make_scaffold_aggregate_fn, scaffold_aggregate_fn
from nvflare_amd.compat import FLModel

pytestmark = pytest.mark.gpu

META, ARRAYS = load_scaffold_golden()
CASES = [c for c in META["cases"] if "expected" in c]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_scaffold_matches_reference(case):
    check_scaffold_result(case, ARRAYS, scaffold_aggregate_fn(scaffold_models_from_case(case, ARRAYS, FLModel), device=0))


@pytest.mark.parametrize("case", [c for c in CASES if c["name"] in ("numpy_k20_special", "torch_ragged")],
                         ids=lambda c: c["name"])
def test_scaffold_sharded_matches_reference(case):
    """Three parameter buckets on one device (sharding.ShardedFedAvg): the same bits."""
    fn = make_scaffold_aggregate_fn(devices=[0, 0, 0])
    check_scaffold_result(case, ARRAYS, fn(scaffold_models_from_case(case, ARRAYS, FLModel)))


def test_controls_add_no_launches():
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    case = next(c for c in CASES if c["name"] == "numpy_full")
    models = scaffold_models_from_case(case, ARRAYS, FLModel)
    n0 = ctx.launch_count()
    aggregate_fn(models, device=0)
    n1 = ctx.launch_count()
    scaffold_aggregate_fn(models, device=0)
    n2 = ctx.launch_count()
    assert n2 - n1 == n1 - n0 > 0
