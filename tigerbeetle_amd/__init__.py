"""tigerbeetle_amd — MI355X-native batch-commit engine for TigerBeetle's create_accounts /
create_transfers state-machine path (drop-in for StateMachine.commit).

    include/tbgpu.h                 C ABI (the drop-in boundary)
    tigerbeetle_amd/csrc/           HIP kernels for gfx950 + the ABI implementation
    tigerbeetle_amd/state_machine   host-side mirror of the reference StateMachine interface
    tigerbeetle_amd/types           Account / Transfer layouts and result codes

The engine library is loaded lazily (tigerbeetle_amd._lib.load) so that the layouts and the
build step are importable on a machine without a GPU.
"""
from .types import (ACCOUNT_DTYPE, BATCH_MAX, RESULT_DTYPE, TRANSFER_DTYPE, AccountFlags,  # noqa: F401
                    CreateAccountResult, CreateTransferResult, Operation, TransferFlags)


def StateMachine(*args, **kw):  # noqa: N802 — mirrors the reference type name
    from .state_machine import StateMachine as _SM
    return _SM(*args, **kw)


def Engine(*args, **kw):  # noqa: N802
    from .state_machine import Engine as _E
    return _E(*args, **kw)
