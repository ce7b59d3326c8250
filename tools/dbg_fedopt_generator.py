import sys, numpy as np, torch, copy
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from golden_util import fedopt_model, load_fedopt_golden
from nvflare_amd.app_opt.pt import PTFedOptModelShareableGenerator
from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, ModelLearnableKey, make_model_learnable
META, A = load_fedopt_golden()
case = META["cases"][0]
model = fedopt_model()
model.load_state_dict({k: torch.from_numpy(np.array(A[v], copy=True)) for k, v in case["init"].items()})
print("init loaded", model.lin1.weight.flatten()[:4])
gen = PTFedOptModelShareableGenerator(optimizer_args=copy.deepcopy(case["optimizer_args"]), source_model=model, device="cuda:0")
gen.handle_event(EventType.START_RUN, FLContext())
print("after start", model.lin1.weight.flatten()[:4], model.lin1.weight.device)
w = {k: np.array(A[v], copy=True) for k, v in case["init"].items()}
exp = case["rounds"][0]
diff = {k: np.array(A[v], copy=True) for k, v in exp["diff"].items()}
fl = FLContext(); fl.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
dev = gen.device_optimizer()
print("bound", dev.p[:4], [(s.name, s.offset, s.n) for s in dev.slots])
out = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl)[ModelLearnableKey.WEIGHTS]
k = "lin1.weight"
p0 = A[case["init"][k]].ravel()[:6]; d = A[exp["diff"][k]].ravel()[:6]; ref = A[exp["weights"][k]].ravel()[:6]; got = out[k].ravel()[:6]
print("p0 ", p0); print("d  ", d); print("ref", ref); print("got", got); print("g buf", dev.g[:6]); print("p buf", dev.p[:6])
