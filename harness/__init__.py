"""Measurement harness used by bench.py and the GPU tests: synthetic frames
generated in HBM (synth) and the trivial copy/read kernels that give the
box's speed of light (membench, rwmix).  Test/bench infrastructure, not
the product."""
