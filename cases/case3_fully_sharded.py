# Case 3 (reference: case3_fully_sharded.py; blog https://irhum.github.io/blog/pjit/#full-sharding)
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
      A: (sharded_X, sharded_Y)
      B: (sharded_X, sharded_Y)
      """)

A = jax.device_put(A, sharding)
print("visualize A: ")
jax.debug.visualize_array_sharding(A)

B = jax.device_put(B, sharding)
print("visualize B: ")
jax.debug.visualize_array_sharding(B)

A_0 = np.array(A.device_buffers[0])
assert A_0.shape == (2,4)
print("A_0.shape: ",A_0.shape)
A_4 = np.array(A.device_buffers[4])
print("Are A_0 and A_4 NOT equal? ", (np.array_equal(A_0, A_4)))
B_0 = np.array(B.device_buffers[0])
B_1 = np.array(B.device_buffers[1])
assert B_0.shape == (8,1)
print("B_0.shape: ", B_0.shape)
print("Are B_0 and B_4 equal? ", (np.array_equal(B_0, B_1)))

# Both operands fully sharded: all-gather A over Y and B over X on the
# contraction dim, then every device computes its unique (2,1) block.
C = jax.lax.dot(A,B)
print("visualize C:")
jax.debug.visualize_array_sharding(C)
print("C.shape: ", C.shape)
C_0 = np.array(C.device_buffers[0])
print("C_0.shape: ", C_0.shape)
assert C_0.shape == (2, 1)
C_1 = np.array(C.device_buffers[1])
C_4 = np.array(C.device_buffers[4])

print("All gather happens...")
print("Are C_0 and C_1 NOT equal? ", (np.array_equal(C_0, C_1)))
print("Are C_0 and C_4 NOT equal? ", (np.array_equal(C_0, C_4)))
print("Are C_0 and C NOT equal? ", (np.array_equal(C_0, C)))
if os.environ.get("LJS_PDB") == "1":   # the reference drops into pdb here unconditionally
    import pdb; pdb.set_trace()
