package triton.client.examples;

import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.concurrent.atomic.AtomicLong;

import triton.client.InferInput;
import triton.client.InferRequestedOutput;
import triton.client.InferenceServerClient;
import triton.client.pojo.DataType;

/**
 * Closed-loop load: T threads x N synchronous infers on "simple"; prints
 * QPS and mean / p99 latency (reference examples/SimpleInferPerf.java).
 *   java ... SimpleInferPerf [host:port] [threads=8] [requests_per_thread=1000]
 */
public class SimpleInferPerf {
  public static void main(String[] args) throws Exception {
    String url = args.length > 0 ? args[0] : "localhost:8000";
    int threads = args.length > 1 ? Integer.parseInt(args[1]) : 8;
    int perThread = args.length > 2 ? Integer.parseInt(args[2]) : 1000;
    InferenceServerClient client = new InferenceServerClient(url, 5000, 5000, threads);
    int[] data = new int[16];
    Arrays.fill(data, 3);
    long[][] lat = new long[threads][perThread];
    AtomicLong failures = new AtomicLong();
    List<Thread> workers = new ArrayList<>();
    long t0 = System.nanoTime();
    for (int t = 0; t < threads; t++) {
      final int tid = t;
      Thread w = new Thread(() -> {
        for (int i = 0; i < perThread; i++) {
          long s = System.nanoTime();
          try {
            InferInput in0 = new InferInput("INPUT0", new long[] {1, 16}, DataType.INT32);
            in0.setData(data, true);
            InferInput in1 = new InferInput("INPUT1", new long[] {1, 16}, DataType.INT32);
            in1.setData(data, true);
            client.infer("simple", Arrays.asList(in0, in1), Arrays.asList(new InferRequestedOutput("OUTPUT0")));
          } catch (Exception e) {
            failures.incrementAndGet();
          }
          lat[tid][i] = System.nanoTime() - s;
        }
      });
      workers.add(w);
      w.start();
    }
    for (Thread w : workers) w.join();
    double secs = (System.nanoTime() - t0) / 1e9;
    long[] all = Arrays.stream(lat).flatMapToLong(Arrays::stream).sorted().toArray();
    double mean = Arrays.stream(all).average().orElse(0) / 1e3;
    double p99 = all[(int) Math.min(all.length - 1, Math.ceil(all.length * 0.99) - 1)] / 1e3;
    System.out.printf("requests: %d, failures: %d, QPS: %.1f, avg latency: %.1f us, p99: %.1f us%n", all.length,
        failures.get(), all.length / secs, mean, p99);
    client.close();
    if (failures.get() > 0) System.exit(1);
  }
}
