"""Diagnostic: a 262,144-session template batch on a dropped (closed) hypervisor,
then a 70-session batch on the same shared store — are its rows distinct, and do
the participant rows read back through the columns and through the worker agree
with the session each row was given?"""
import sys

import numpy as np
import torch  # noqa: F401 - loaded before the native extension

sys.path.insert(0, ".")
from agent_hypervisor_amd.models import store_template as TT  # noqa: E402
from hypervisor import Hypervisor  # noqa: E402


def check(hv, n, agents, tag):
    st = hv._store
    sa = np.arange(n) % agents.count
    run = TT.run(hv, n, agents=agents, session_agent=sa, now_us=1767225600123456)
    b = hv._sessions.batch_of(run.session_ids[0])
    slots = b.slots.astype(np.int64)
    dup = len(slots) - len(np.unique(slots))
    g = st.gather({"p_agent": slots})  # participant 0 plane: row = slot
    exp = agents.agent_id.cpu().numpy()[sa]
    col_bad = np.flatnonzero(g["p_agent"] != exp)
    view_bad = []
    for i in range(n):
        m = hv.get_session(run.session_ids[i])
        ps = list(m.sso._participants)
        if ps != [agents.dids[sa[i]]]:
            view_bad.append((i, ps))
    print(tag, "dup slots", dup, "column mismatches", col_bad[:10].tolist(), "view mismatches", view_bad[:5],
          "slots", slots[:8].tolist(), flush=True)
    return run


hv1 = Hypervisor(device="cuda")
big = TT.AgentSet.synthetic(hv1._store, 4096, seed=11, prefix="did:mesh:diag-agent-")
r1 = TT.run(hv1, 262144, agents=big, variant=(3, 0))
for sid in r1.session_ids[:8]:
    hv1.get_session(sid)
st = hv1._store
print("live before close", st.live_rows(), flush=True)
del hv1, r1
print("live after close", st.live_rows(), flush=True)
hv2 = Hypervisor(device="cuda")
agents = TT.AgentSet(st, [f"did:mesh:tmpl-agent-{k}" for k in range(7)] + ["did:x"],
                     [0.8, 0.3, 0.61, 0.96, 0.6, 0.95, 0.05, 0.7])
check(hv2, 70, agents, "after-close")
hv3 = Hypervisor(device="cuda")
check(hv3, 70, agents, "again")
