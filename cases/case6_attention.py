# GSPMD paper (https://arxiv.org/pdf/2105.04663.pdf) section 5.1, Figure 7 (reference: case6_attention.py)
import os
os.environ["XLA_FLAGS"] = '--xla_force_host_platform_device_count=4'
os.environ.setdefault("LJS_NUM_DEVICES", "4")   # 4 virtual devices when run on one MI355X
# On a node with >= 4 MI355X the same 4 devices are 4 physical GPUs driven by this one process
# (the reference's single-controller model): mesh-axis collectives become grouped RCCL calls over
# xGMI (comm/native.py, ncclCommInitAll + ncclCommSplit per group).  Such single-controller steps
# run eagerly unless LJS_MULTI_GPU_CAPTURE=1 captures them as ONE multi-device HIP graph
# (spmd/graphs.py MultiDeviceGraph); torchrun + bench.py is the captured one-process-per-GPU path.

import functools
import numpy as np
import learning_jax_sharding_amd as jax
import learning_jax_sharding_amd.numpy as jnp
from learning_jax_sharding_amd.experimental import mesh_utils
from learning_jax_sharding_amd.sharding import PartitionSpec, NamedSharding
from learning_jax_sharding_amd.sharding import Mesh

from learning_jax_sharding_amd import nn
from learning_jax_sharding_amd.training import train_state
from learning_jax_sharding_amd.nn import partitioning as nn_partitioning
from learning_jax_sharding_amd import optim as optax

import time

# Input (B,S,M): y = Attention(Wq x, Wk x, Wv x) Wo; Wq/Wk/Wv project to (B,S,N,D), Wo back to (B,S,M).
# Feed-forward: y = Relu(Win x) Wout (learning_jax_sharding_amd.nn.FeedForward).

ATTN_IMPL = os.environ.get("ATTN_IMPL", "fused")  # "fused" HIP flash attention | "einsum" (reference form)


class FlaxAttention(nn.Module):
  query_dim: int
  heads: int = 8
  dim_head: int = 64
  dropout: float = 0.0
  dtype: jnp.dtype = jnp.bfloat16

  def setup(self):
    inner_dim = self.dim_head * self.heads
    self.scale = self.dim_head ** -0.5

    # Wq, Wk, Wv.  Shape: MND.  Shardings: X,Y,_
    qkv_init_kernel = nn.with_logical_partitioning(
      nn.initializers.lecun_normal(),
      ('embed','heads')
    )
    self.query = nn.Dense(inner_dim, kernel_init=qkv_init_kernel, use_bias=False, dtype=self.dtype, name="to_q")
    self.key = nn.Dense(inner_dim, kernel_init=qkv_init_kernel, use_bias=False, dtype=self.dtype, name="to_k")
    self.value = nn.Dense(inner_dim, kernel_init=qkv_init_kernel, use_bias=False, dtype=self.dtype, name="to_v")
    self.proj_attn = nn.Dense(
        self.query_dim,
        kernel_init=nn.with_logical_partitioning(nn.initializers.lecun_normal(), ('heads','embed')),
        dtype=self.dtype,
        name="to_out_0")
    self.dropout_layer = nn.Dropout(rate=self.dropout)

  def __call__(self, hidden_states, context=None, deterministic=True):
    context = hidden_states if context is None else context
    print("context.shape: ", context.shape)
    if context is hidden_states:
      # Q/K/V projections as ONE batched MFMA GEMM over the three kernels
      m = hidden_states.shape[-1]
      query_proj, key_proj, value_proj = jax.ops.dense(
          hidden_states, [self.query.kernel_param(m), self.key.kernel_param(m), self.value.kernel_param(m)],
          None, compute_dtype=self.dtype)
    else:
      query_proj = self.query(hidden_states)
      key_proj = self.key(context)
      value_proj = self.value(context)
    print("query_proj.shape: ", query_proj.shape)

    # heads is replicated, so the head split below moves no data
    query_proj = nn.with_logical_constraint(query_proj, ('batch', 'embed', None))
    key_proj = nn.with_logical_constraint(key_proj, ('batch', 'embed', None))
    value_proj = nn.with_logical_constraint(value_proj, ('batch', 'embed', None))

    b = hidden_states.shape[0]
    query_states = jnp.reshape(query_proj, (b, -1, self.heads, self.dim_head))
    key_states = jnp.reshape(key_proj, (b, -1, self.heads, self.dim_head))
    value_states = jnp.reshape(value_proj, (b, -1, self.heads, self.dim_head))

    query_states = nn.with_logical_constraint(query_states, ('batch', 'embed', None, None))
    key_states = nn.with_logical_constraint(key_states, ('batch', 'embed', None, None))
    value_states = nn.with_logical_constraint(value_states, ('batch', 'embed', None, None))

    print("query_states.shape: ", query_states.shape)

    if ATTN_IMPL == "einsum":
      # Attn stability: f32 Q/K, f32 softmax, bf16 probabilities
      query_states = jnp.float32(query_states)
      key_states = jnp.float32(key_states)
      attention_scores = jnp.einsum("b t n h, b f n h -> b n f t", key_states, query_states)
      attention_scores = attention_scores * self.scale
      attention_probs = nn.softmax(attention_scores, axis=-1)
      attention_probs = jnp.asarray(attention_probs, dtype=self.dtype)
      hidden_states = jnp.einsum("b n f t, b t n h -> b f n h", attention_probs, value_states)
    else:
      # the same math as one fused HIP kernel (QK^T -> scale -> f32 softmax -> bf16 P -> PV)
      hidden_states = jax.ops.dot_product_attention(query_states, key_states, value_states, self.scale)
    b = hidden_states.shape[0]
    hidden_states = jnp.reshape(hidden_states, (b, -1, self.heads * self.dim_head))

    hidden_states = nn.with_logical_constraint(hidden_states, ('batch', 'kv', 'heads'))

    hidden_states = self.proj_attn(hidden_states)

    hidden_states = nn.with_logical_constraint(hidden_states,('batch', 'embed'))

    return self.dropout_layer(hidden_states, deterministic=deterministic)

# 2D finalized

key = jax.random.key(0)

B = 8
S = 256
M = 640
x = jax.random.normal(key, (B,S,M))

# Create mesh
device_mesh = mesh_utils.create_device_mesh((2, 2))
mesh = Mesh(devices=device_mesh, axis_names=('data','model'))

def mesh_sharding(pspec: PartitionSpec) -> NamedSharding:
  return NamedSharding(mesh, pspec)
# Data sharding
x_sharding = mesh_sharding(PartitionSpec('data', 'model'))
x = jax.device_put(x, x_sharding)
print("Visualize x[0]: ")
jax.debug.visualize_array_sharding(x[0])
x_0 = x.device_buffers[0]
print("x[0] shape: ", x_0.shape)

attention = FlaxAttention(M)

def init_fn(k, x, model, optimizer):
  variables = model.init(k, x)
  state = train_state.TrainState.create(
    apply_fn=model.apply,
    params=variables['params'],
    tx=optimizer
  )
  return state

init_rngs = {'params' : jax.random.PRNGKey(1), 'dropout' : jax.random.PRNGKey(2)}
optimizer = optax.adam(learning_rate=0.001)

rules = (
  ('batch', 'data'),
  ('embed', 'model'),
  ('hidden', 'model'),
)
# LJS_RULES=gspmd2d runs the "2D finalized" layout of the comment above (embed->data,
# heads->model: Wq_0 is (320, 256)); megatron / fsdp are the other presets
if os.environ.get("LJS_RULES"):
  from learning_jax_sharding_amd import parallel
  rules = parallel.rules(os.environ["LJS_RULES"])

logical_abstract_variables = jax.eval_shape(functools.partial(init_fn, model=attention, optimizer=optimizer), init_rngs, x)
logical_state_spec = nn.get_partition_spec(logical_abstract_variables)
logical_state_sharding = nn.logical_to_mesh_sharding(logical_state_spec, mesh, rules)
jit_init_fn = jax.jit(init_fn, static_argnums=(2,3),
                      in_shardings=(mesh_sharding(None), x_sharding),
                      out_shardings=logical_state_sharding)

initialized_state = jit_init_fn(init_rngs,x,attention, optimizer)
print("Visualize Wq sharding:")
jax.debug.visualize_array_sharding(initialized_state.params['to_q']['kernel'].value)
to_q = initialized_state.params['to_q']['kernel'].value
to_q_0 = to_q.device_buffers[0]
print("Wq shape: ", )
print("Wq shape: ", to_q.shape)
print("Wq_0 shape: ", to_q_0.shape)
print("x[0] shape: ", x_0.shape)

@functools.partial(jax.jit, in_shardings=(logical_state_sharding, x_sharding),
                   out_shardings=logical_state_sharding)
def train_step(state, x):
  def loss_unrolled(params):
    y = attention.apply({'params' : params}, x)
    return y.sum()
  grad_fn = jax.grad(loss_unrolled)
  grads = grad_fn(state.params)
  state = state.apply_gradients(grads=grads)
  return state

with mesh, nn_partitioning.axis_rules(rules):
  new_state = train_step(initialized_state, x)

# With the reference rules x[0] is (4, 128, 640) and Wq[0] is (320, 512): 'heads' has no rule,
# so the projection's output dim stays replicated.  The reference's comment expects (320, 256):
# that is the GSPMD-paper 2D layout (embed->data, heads->model), LJS_RULES=gspmd2d.

@functools.partial(jax.jit, in_shardings=(logical_state_sharding, x_sharding),
                   out_shardings=x_sharding)
def apply_fn(state, x):
  return state.apply_fn({"params" : state.params}, x)

with mesh, nn_partitioning.axis_rules(rules):
  s = time.time()
  for i in range(10):
    y = apply_fn(new_state, x)
  print("time for 10 itters: ", (time.time() - s))
