import sys, numpy as np
sys.path.insert(0, ".")
from tigerbeetle_amd.state_machine import Engine, Options
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, TransferFlags
for mode in ("commit", "pipelined", "noset"):
    e = Engine(Options(accounts_max=4096, transfers_max=1 << 17, pass_events_max=8192 * 4, pass_batches_max=64))
    acc = np.zeros(2, dtype=ACCOUNT_DTYPE); acc["id_lo"]=[1,2]; acc["ledger"]=1; acc["code"]=1
    print(mode, e.commit(128,10,acc.tobytes()))
    pend=np.zeros(1,dtype=TRANSFER_DTYPE); pend["id_lo"]=10; pend["debit_account_id_lo"]=1; pend["credit_account_id_lo"]=2; pend["amount_lo"]=100; pend["ledger"]=1; pend["code"]=1; pend["flags"]=int(TransferFlags.pending)
    print(e.commit(129,20,pend.tobytes()))
    if mode != "noset":
        e.set_balances(1,0,0,0,0)
    print("accounts", e.export_accounts()[["id_lo","debits_pending_lo","credits_pending_lo"]])
    x=np.zeros(1,dtype=TRANSFER_DTYPE); x["id_lo"]=11; x["pending_id_lo"]=10; x["flags"]=int(TransferFlags.post_pending_transfer); x["ledger"]=1; x["code"]=1
    try:
        if mode == "pipelined":
            rb, rep, _ = e.commit_pipelined(129, [30], [1], np.frombuffer(x.tobytes(), dtype=np.uint8).copy(), chunk_batches=1)
            print("pipelined rb", rb, rep[:8])
        else:
            print("reply", e.commit(129,30,x.tobytes()))
    except Exception as ex: print("raised", ex)
    print("stats", {k: v for k, v in e.stats().items() if k in ("dependent_events", "passes")})
    e.close()
