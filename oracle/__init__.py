"""Test infrastructure only: the CPU restatement (oracle) and the reference drivers (_ref)."""
