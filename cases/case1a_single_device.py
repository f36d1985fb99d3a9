# Case 1a on a 1-device CPU mesh: the "plumbing" config of BASELINE.json ("case1a replicated
# matmul on a 1-device CPU mesh").  Same program as case1a.py (reference case1a.py:15-62) with
# the device grid shrunk to (1, 1): every placement is whole-array, the dot needs no
# collective, and every buffer equals the global array.
import os
os.environ["XLA_FLAGS"] = '--xla_force_host_platform_device_count=1'
os.environ.setdefault("LJS_PLATFORM", "cpu")
os.environ.setdefault("LJS_NUM_DEVICES", "1")
import numpy as np
import learning_jax_sharding_amd as jax
from learning_jax_sharding_amd.experimental import mesh_utils
from learning_jax_sharding_amd.sharding import PositionalSharding
from learning_jax_sharding_amd.spmd import plan as _plan

print("""
Case 1a on one device.
      A: (full, full)
      B: (full, full)
      """)

sharding = PositionalSharding(mesh_utils.create_device_mesh((1,1)))
key = jax.random.PRNGKey(0)
A = jax.random.normal(key, (4, 16))
B = jax.random.normal(key, (16, 4))

A = jax.device_put(A, sharding.replicate(axis=0, keepdims=True))
print("A:")
jax.debug.visualize_array_sharding(A)

B = jax.device_put(B, sharding.reshape(1,1).replicate(axis=1, keepdims=True))
print("B:")
jax.debug.visualize_array_sharding(B)

A_0 = np.array(A.device_buffers[0])
assert A_0.shape == (4,16)
print("A_0.shape: ",A_0.shape)
print("Is A_0 equal to A? ", (np.array_equal(A_0, A)))

B_0 = np.array(B.device_buffers[0])
assert B_0.shape == (16,4)
print("B_0.shape: ", B_0.shape)
print("Are A and B the same numbers? ", (np.array_equal(np.array(A).ravel(), np.array(B).ravel())))

with _plan.record_plan() as rec:
  C = jax.lax.dot(A,B)
print("C:")
jax.debug.visualize_array_sharding(C)
print("collectives: ", rec.collective_kinds())

C_0 = np.array(C.device_buffers[0])
print("C_0.shape: ", C_0.shape)
print("Number of buffers: ", len(C.device_buffers))
print("Are C_0 and C equal? ", (np.array_equal(C_0, C)))
print("Is C == A @ B? ", bool(np.allclose(C_0, np.array(A) @ np.array(B), rtol=1e-5, atol=1e-5)))
