# Case 1a (reference: case1a.py; blog https://irhum.github.io/blog/pjit/#case-1a-mesh-axes-match)
# Contraction dim sharded on both operands; result replicated via all-reduce.
import os
os.environ["XLA_FLAGS"] = '--xla_force_host_platform_device_count=8'
os.environ.setdefault("LJS_NUM_DEVICES", "8")   # 8 virtual devices when run on one MI355X
import numpy as np
import learning_jax_sharding_amd as jax
from learning_jax_sharding_amd.experimental import mesh_utils
from learning_jax_sharding_amd.sharding import PositionalSharding

print("""
This is the case for AllGather.
      A: (full, sharded)
      B: (sharded, full)
      """)

sharding = PositionalSharding(mesh_utils.create_device_mesh((2,4)))
key = jax.random.PRNGKey(0)
A = jax.random.normal(key, (4, 16))
B = jax.random.normal(key, (16, 4))

# A: inner (contraction) axis sharded over Y, replicated over X.
A = jax.device_put(A, sharding.replicate(axis=0, keepdims=True))
print("A:")
jax.debug.visualize_array_sharding(A)

# B: the (2,4) grid reshaped to (4,2), replicated over its second axis: contraction block d//2.
B = jax.device_put(B, sharding.reshape(4,2).replicate(axis=1, keepdims=True))
print("B:")
jax.debug.visualize_array_sharding(B)

A_0 = np.array(A.device_buffers[0])
assert A_0.shape == (4,4)
print("A_0.shape: ",A_0.shape)

A_4 = np.array(A.device_buffers[4])
print("Are A_0 and A_4 equal? ", (np.array_equal(A_0, A_4)))

B_0 = np.array(B.device_buffers[0])
assert B_0.shape == (4,4)
B_1 = np.array(B.device_buffers[1])
print("B_0.shape: ", B_0.shape)
print("Are B_0 and B_4 equal? ", (np.array_equal(B_0, B_1)))

# A's contraction blocks follow d%4, B's follow d//2: the partitioner permutes B,
# does the local (4,4)@(4,4) dot and all-reduces the partial sums over Y.
C = jax.lax.dot(A,B)
print("C:")
jax.debug.visualize_array_sharding(C)

C_0 = np.array(C.device_buffers[0])
C_1 = np.array(C.device_buffers[1])
C_4 = np.array(C.device_buffers[4])

print("All reduce happens...")
print("Are C_0 and C_1 equal? ", (np.array_equal(C_0, C_1)))
print("Are C_0 and C_4 equal? ", (np.array_equal(C_0, C_4)))
print("Are C_0 and C equal? ", (np.array_equal(C_0, C)))
