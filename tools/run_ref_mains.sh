mkdir -p gpurun_out/mains; cd physics-llm-inference_amd
for m in ch06.flash_attention ch06.attention_memory ch06.online_softmax ch09.nccl_primitives ch09.tensor_parallel ch05.tensor_cores ch05.triton_matmul ch05.shared_memory ch08.cuda_graph ch02.cached_generation ch09.moe_layer; do
  timeout -k 10 200 python3 -u -m $m > ../gpurun_out/mains/$m.txt 2>&1 || { echo "FAIL $m"; exit 1; }
done
