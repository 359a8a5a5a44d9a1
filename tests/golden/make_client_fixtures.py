"""Writes tests/golden/client_known_answers.json: the known answers of the reference's client
integration tests, transcribed as data.

The scenarios are the server-side steps of:
  * Java  src/clients/java/src/test/java/com/tigerbeetle/IntegrationTest.java:29-70 (the two
    accounts and their ids) and :699-781 (testCreateLinkedTransfers: a linked pair 100 / 49, the
    balances 100 / 49 on both sides, both transfers found with a non-zero timestamp);
  * Node  src/clients/node/src/test.ts:19-47 (accounts A = 17, B = 19) and :68-341 (create, the
    `exists` error, lookups, a transfer, a two-phase transfer posted, one voided, and a linked pair
    whose second member repeats the first's id: linked_event_failed + exists_with_different_flags).
Client-side checks (the u16 range check of `code`, the client refusing a non-zero timestamp) never
reach the state machine and are left out.

Every field value, expected result and expected balance below is copied from those assertions;
nothing is computed.  Run from the repo root: python tests/golden/make_client_fixtures.py
"""
import json
import os

JAVA = "src/clients/java/src/test/java/com/tigerbeetle/IntegrationTest.java"
NODE = "src/clients/node/src/test.ts"

# IntegrationTest.java:37-61: account ids are little-endian byte arrays {1, 0, ...} and {2, 0, ...};
# setUserData128(100, 0) is (least, most significant).
JAVA_ACCOUNTS = [
    dict(id=1, user_data_128=100, user_data_64=101, user_data_32=102, ledger=720, code=1),
    dict(id=2, user_data_128=200, user_data_64=201, user_data_32=202, ledger=720, code=2),
]
LINKED = 1
PENDING = 2
POST = 4
VOID = 8

java = {
    "name": "java_create_linked_transfers",
    "source": JAVA + ":29-70,699-781",
    "steps": [
        {"op": "create_accounts", "events": JAVA_ACCOUNTS, "results": []},
        {"op": "create_transfers", "events": [
            dict(id=10, credit_account_id=1, debit_account_id=2, ledger=720, code=1, amount=100, flags=LINKED),
            dict(id=20, credit_account_id=2, debit_account_id=1, ledger=720, code=1, amount=49, flags=0),
        ], "results": []},
        {"op": "lookup_accounts", "ids": [1, 2], "expect": [
            dict(JAVA_ACCOUNTS[0], flags=0, credits_posted=100, debits_posted=49, credits_pending=0, debits_pending=0,
                 timestamp_nonzero=True),
            dict(JAVA_ACCOUNTS[1], flags=0, credits_posted=49, debits_posted=100, credits_pending=0, debits_pending=0,
                 timestamp_nonzero=True),
        ]},
        {"op": "lookup_transfers", "ids": [10, 20], "expect": [
            dict(id=10, credit_account_id=1, debit_account_id=2, ledger=720, code=1, amount=100, flags=LINKED,
                 timestamp_nonzero=True),
            dict(id=20, credit_account_id=2, debit_account_id=1, ledger=720, code=1, amount=49, flags=0,
                 timestamp_nonzero=True),
        ]},
    ],
}

# test.ts:19-47.
A = dict(id=17, user_data_128=0, user_data_64=0, user_data_32=0, ledger=1, code=718, flags=0)
B = dict(id=19, user_data_128=0, user_data_64=0, user_data_32=0, ledger=1, code=719, flags=0)


def balances(acct, dp, dpost, cp, cpost):
    return dict(acct, debits_pending=dp, debits_posted=dpost, credits_pending=cp, credits_posted=cpost,
                timestamp_nonzero=True)


node = {
    "name": "node_client_flow",
    "source": NODE + ":19-47,68-341",
    "steps": [
        # :68-71 can create accounts
        {"op": "create_accounts", "events": [A], "results": []},
        # :73-78 can return error on account
        {"op": "create_accounts", "events": [A, B], "results": [[0, "exists"]]},
        # :85-118 can lookup accounts
        {"op": "lookup_accounts", "ids": [17, 19], "expect": [balances(A, 0, 0, 0, 0), balances(B, 0, 0, 0, 0)]},
        # :120-155 can create a transfer
        {"op": "create_transfers", "events": [
            dict(id=1, debit_account_id=19, credit_account_id=17, amount=100, ledger=1, code=1, flags=0)],
         "results": []},
        {"op": "lookup_accounts", "ids": [17, 19], "expect": [balances(A, 0, 0, 0, 100), balances(B, 0, 100, 0, 0)]},
        # :157-205 can create a two-phase transfer
        {"op": "create_transfers", "events": [
            dict(id=2, debit_account_id=19, credit_account_id=17, amount=50, timeout=2000000000, ledger=1, code=1,
                 flags=PENDING)], "results": []},
        {"op": "lookup_accounts", "ids": [17, 19], "expect": [balances(A, 0, 0, 50, 100), balances(B, 50, 100, 0, 0)]},
        {"op": "lookup_transfers", "ids": [2], "expect": [
            dict(id=2, debit_account_id=19, credit_account_id=17, amount=50, user_data_128=0, user_data_64=0,
                 user_data_32=0, code=1, flags=2, timeout_nonzero=True, timestamp_nonzero=True)]},
        # :207-238 can post a two-phase transfer
        {"op": "create_transfers", "events": [
            dict(id=3, debit_account_id=0, credit_account_id=0, amount=0, pending_id=2, ledger=1, code=1, flags=POST)],
         "results": []},
        {"op": "lookup_accounts", "ids": [17, 19], "expect": [balances(A, 0, 0, 0, 150), balances(B, 0, 150, 0, 0)]},
        # :240-290 can reject a two-phase transfer
        {"op": "create_transfers", "events": [
            dict(id=4, debit_account_id=19, credit_account_id=17, amount=50, timeout=1000000000, ledger=1, code=1,
                 flags=PENDING)], "results": []},
        {"op": "create_transfers", "events": [
            dict(id=5, debit_account_id=0, credit_account_id=0, amount=0, pending_id=4, ledger=1, code=1, flags=VOID)],
         "results": []},
        {"op": "lookup_accounts", "ids": [17, 19], "expect": [balances(A, 0, 0, 0, 150), balances(B, 0, 150, 0, 0)]},
        # :292-341 can link transfers
        {"op": "create_transfers", "events": [
            dict(id=6, debit_account_id=19, credit_account_id=17, amount=100, ledger=1, code=1, flags=LINKED),
            dict(id=6, debit_account_id=19, credit_account_id=17, amount=100, ledger=1, code=1, flags=0)],
         "results": [[0, "linked_event_failed"], [1, "exists_with_different_flags"]]},
        {"op": "lookup_accounts", "ids": [17, 19], "expect": [balances(A, 0, 0, 0, 150), balances(B, 0, 150, 0, 0)]},
    ],
}


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "client_known_answers.json")
    with open(out, "w") as f:
        json.dump({"generated_by": "tests/golden/make_client_fixtures.py", "scenarios": [java, node]}, f, indent=1)
        f.write("\n")
    print(out)


if __name__ == "__main__":
    main()
