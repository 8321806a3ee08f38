"""CPU baseline leg of bench.py -- TEST/BENCH INFRASTRUCTURE ONLY (see oracle/bls_oracle.py header)."""


def measure_same_message(sample=None):
    return None
