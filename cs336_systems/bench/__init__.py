"""Benchmark / profiling drivers (reference L4 harness): ``e2e`` (model step timing +
memory), ``attention`` (naive vs FlashAttention sweeps), ``flash`` (FA2 TFLOPS / leaderboard),
``collectives`` (RCCL all-reduce microbenchmark), ``ddp`` (DP-variant training driver),
``precision`` (mixed-precision demos)."""
