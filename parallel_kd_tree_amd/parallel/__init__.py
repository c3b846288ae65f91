"""Multi-GPU decompositions over torch.distributed (backend "nccl" = RCCL over xGMI)."""
