"""Import-path alias kept for drop-in compatibility with `from ops.triton.jagged import ...`.
There is no Triton in this build: the implementation is the HIP path in ops/jagged.py."""
