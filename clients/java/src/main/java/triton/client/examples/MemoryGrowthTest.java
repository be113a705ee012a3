package triton.client.examples;

import java.util.Arrays;

import triton.client.InferInput;
import triton.client.InferRequestedOutput;
import triton.client.InferResult;
import triton.client.InferenceServerClient;
import triton.client.pojo.DataType;

/**
 * Repeated large requests through one client while watching heap use: the
 * used heap after the run must stay within a bound of the warm-up level
 * (reference examples/MemoryGrowthTest.java).
 *   java ... MemoryGrowthTest [host:port] [iterations=1000]
 */
public class MemoryGrowthTest {
  private static long usedHeap() {
    Runtime rt = Runtime.getRuntime();
    System.gc();
    return rt.totalMemory() - rt.freeMemory();
  }

  public static void main(String[] args) throws Exception {
    String url = args.length > 0 ? args[0] : "localhost:8000";
    int iters = args.length > 1 ? Integer.parseInt(args[1]) : 1000;
    float[] payload = new float[1 << 18];  // 1 MiB FP32 tensor
    for (int i = 0; i < payload.length; i++) payload[i] = i % 97;
    try (InferenceServerClient client = new InferenceServerClient(url, 5000, 30000)) {
      long warm = 0;
      for (int it = 0; it < iters; it++) {
        InferInput in = new InferInput("INPUT0", new long[] {payload.length}, DataType.FP32);
        in.setData(payload, true);
        InferResult r = client.infer("identity_fp32", Arrays.asList(in),
            Arrays.asList(new InferRequestedOutput("OUTPUT0", true)));
        float[] out = r.getOutputAsFloat("OUTPUT0");
        if (out.length != payload.length || out[payload.length - 1] != payload[payload.length - 1]) {
          System.err.println("error: wrong identity output");
          System.exit(1);
        }
        if (it == 10) warm = usedHeap();
      }
      long end = usedHeap();
      System.out.printf("heap after warm-up %d KiB, after %d iterations %d KiB%n", warm >> 10, iters, end >> 10);
      if (end > warm + (64L << 20)) {
        System.err.println("error: heap grew by more than 64 MiB");
        System.exit(1);
      }
    }
    System.out.println("PASS: memory growth");
  }
}
