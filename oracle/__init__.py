"""CPU oracle for the MI355X realtime style-transfer path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package. See numpy_ref.py for
the reference file:line map and the parity-pinning status.
"""
