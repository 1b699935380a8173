"""CPU oracle for parity tests — TEST INFRASTRUCTURE ONLY (see oracle/unet_ref.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
"""
