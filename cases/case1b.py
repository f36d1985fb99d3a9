# Case 1b (reference: case1b.py; blog https://irhum.github.io/blog/pjit/#case-1b-mesh-axes-mismatch)
import os
os.environ["XLA_FLAGS"] = '--xla_force_host_platform_device_count=8'
os.environ.setdefault("LJS_NUM_DEVICES", "8")
import numpy as np
import learning_jax_sharding_amd as jax
from learning_jax_sharding_amd.experimental import mesh_utils
from learning_jax_sharding_amd.sharding import PositionalSharding

sharding = PositionalSharding(mesh_utils.create_device_mesh((2,4)))
key = jax.random.PRNGKey(0)
A = jax.random.normal(key, (4, 16))
B = jax.random.normal(key, (16, 4))

print("""
This is the case for AllReduce.
      A: (full, shardedY)
      B: (shardedX, full)
      """)

A = jax.device_put(A, sharding.replicate(axis=0, keepdims=True))
print("visualize A: ")
jax.debug.visualize_array_sharding(A)

B = jax.device_put(B, sharding.replicate(axis=1, keepdims=True))
print("visualize B: ")
jax.debug.visualize_array_sharding(B)

A_0 = np.array(A.device_buffers[0])
assert A_0.shape == (4,4)
print("A_0.shape: ",A_0.shape)
A_4 = np.array(A.device_buffers[4])
print("Are A_0 and A_4 equal? ", (np.array_equal(A_0, A_4)))
B_0 = np.array(B.device_buffers[0])
B_1 = np.array(B.device_buffers[1])
assert B_0.shape == (8,4)
print("B_0.shape: ", B_0.shape)
print("Are B_0 and B_4 equal? ", (np.array_equal(B_0, B_1)))

C = jax.lax.dot(A,B)
print("visualize C:")
jax.debug.visualize_array_sharding(C)
print("C.shape: ", C.shape)
C_0 = np.array(C.device_buffers[0])
C_1 = np.array(C.device_buffers[1])
C_4 = np.array(C.device_buffers[4])

print("All gather happens...")
print("Are C_0 and C_1 equal? ", (np.array_equal(C_0, C_1)))
print("Are C_0 and C_4 equal? ", (np.array_equal(C_0, C_4)))
print("Are C_0 and C equal? ", (np.array_equal(C_0, C)))
