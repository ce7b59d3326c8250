"""CPU oracle for the FedAvg hot path -- test infrastructure only (see fedavg_oracle.py header)."""
