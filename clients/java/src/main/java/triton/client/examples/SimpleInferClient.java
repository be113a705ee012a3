package triton.client.examples;

import java.util.Arrays;
import java.util.List;

import triton.client.InferInput;
import triton.client.InferRequestedOutput;
import triton.client.InferResult;
import triton.client.InferenceServerClient;
import triton.client.pojo.DataType;

/**
 * add/sub on the "simple" model, once with binary tensors and once with
 * JSON data (reference examples/SimpleInferClient.java).
 *   java -cp triton-client.jar triton.client.examples.SimpleInferClient [host:port]
 */
public class SimpleInferClient {
  public static void main(String[] args) throws Exception {
    String url = args.length > 0 ? args[0] : "localhost:8000";
    int[] a = new int[16];
    int[] b = new int[16];
    for (int i = 0; i < 16; i++) {
      a[i] = i;
      b[i] = 1;
    }
    try (InferenceServerClient client = new InferenceServerClient(url, 5000, 5000)) {
      if (!client.isServerLive()) throw new IllegalStateException("server is not live");
      for (boolean isBinary : new boolean[] {true, false}) {
        InferInput in0 = new InferInput("INPUT0", new long[] {1, 16}, DataType.INT32);
        in0.setData(a, isBinary);
        InferInput in1 = new InferInput("INPUT1", new long[] {1, 16}, DataType.INT32);
        in1.setData(b, isBinary);
        List<InferRequestedOutput> outputs = Arrays.asList(
            new InferRequestedOutput("OUTPUT0", isBinary), new InferRequestedOutput("OUTPUT1", isBinary));
        InferResult r = client.infer("simple", Arrays.asList(in0, in1), outputs);
        int[] sum = r.getOutputAsInt("OUTPUT0");
        int[] diff = r.getOutputAsInt("OUTPUT1");
        for (int i = 0; i < 16; i++) {
          System.out.println(a[i] + " + " + b[i] + " = " + sum[i] + "; " + a[i] + " - " + b[i] + " = " + diff[i]);
          if (sum[i] != a[i] + b[i] || diff[i] != a[i] - b[i]) {
            System.err.println("error: incorrect result");
            System.exit(1);
          }
        }
      }
    }
    System.out.println("PASS: infer");
  }
}
