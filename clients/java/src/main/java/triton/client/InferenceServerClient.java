package triton.client;

import java.io.ByteArrayOutputStream;
import java.io.IOException;
import java.net.URI;
import java.net.URLEncoder;
import java.net.http.HttpClient;
import java.net.http.HttpRequest;
import java.net.http.HttpResponse;
import java.nio.charset.StandardCharsets;
import java.time.Duration;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.concurrent.CompletableFuture;
import java.util.concurrent.CompletionException;
import java.util.concurrent.ExecutorService;
import java.util.concurrent.Executors;

import triton.client.endpoint.AbstractEndpoint;
import triton.client.endpoint.FixedEndpoint;
import triton.client.pojo.IOTensor;
import triton.client.pojo.Json;
import triton.client.pojo.Parameters;

/**
 * KServe-v2 HTTP/REST inference client (reference
 * src/java/src/main/java/triton/client/InferenceServerClient.java:73-470).
 *
 * Same surface as the reference subset (sync {@link #infer}, retries,
 * per-request headers / query params, {@link InferArguments}) plus
 * {@link #inferAsync} and the health/metadata calls. Built on the JDK's
 * {@code java.net.http.HttpClient} (HTTP/1.1 keep-alive pool), so the
 * library needs no third-party jars.
 */
public class InferenceServerClient implements AutoCloseable {
  private static final String HEADER_LEN = "Inference-Header-Content-Length";

  /** Connection / timeout settings (reference HttpConfig, :80-165). */
  public static class HttpConfig {
    private int ioThreadNum = Math.max(2, Runtime.getRuntime().availableProcessors());
    private int readTimeout = 10000;
    private int connectTimeout = 5000;
    private int maxConnectionCount = 100;
    private int maxConnectionPerRoute = 100;
    private int requestTimeout = 10000;
    private boolean keepAlive = true;

    public HttpConfig() {}

    public HttpConfig(int connectTimeout, int readTimeout) {
      this.connectTimeout = connectTimeout;
      this.readTimeout = readTimeout;
    }

    public HttpConfig(int ioThreadNum, int connectTimeout, int readTimeout, int requestTimeout) {
      this(connectTimeout, readTimeout);
      this.ioThreadNum = ioThreadNum;
      this.requestTimeout = requestTimeout;
    }

    public int getIoThreadNum() { return ioThreadNum; }

    public void setIoThreadNum(int n) {
      Util.checkArgument(n > 0, "ioThreadNum must be > 0");
      ioThreadNum = n;
    }

    public int getReadTimeout() { return readTimeout; }

    public void setReadTimeout(int ms) {
      Util.checkArgument(ms > 0, "readTimeout must be > 0");
      readTimeout = ms;
    }

    public int getConnectTimeout() { return connectTimeout; }

    public void setConnectTimeout(int ms) {
      Util.checkArgument(ms > 0, "connectTimeout must be > 0");
      connectTimeout = ms;
    }

    public int getMaxConnectionCount() { return maxConnectionCount; }

    public void setMaxConnectionCount(int n) { maxConnectionCount = n; }

    public int getMaxConnectionPerRoute() { return maxConnectionPerRoute; }

    public void setMaxConnectionPerRoute(int n) { maxConnectionPerRoute = n; }

    public int getRequestTimeout() { return requestTimeout; }

    public void setRequestTimeout(int ms) { requestTimeout = ms; }

    public boolean isKeepAlive() { return keepAlive; }

    public void setKeepAlive(boolean keepAlive) { this.keepAlive = keepAlive; }
  }

  private final AbstractEndpoint endpoint;
  private final HttpConfig config;
  private final ExecutorService executor;
  private final HttpClient http;
  private int retryCnt = 3;

  public InferenceServerClient(String endpoint, int connectTimeout, int readTimeout) {
    this(new FixedEndpoint(endpoint), new HttpConfig(connectTimeout, readTimeout));
  }

  public InferenceServerClient(String endpoint, int connectTimeout, int readTimeout, int ioThreadNum) {
    this(new FixedEndpoint(endpoint), new HttpConfig(ioThreadNum, connectTimeout, readTimeout, readTimeout));
  }

  public InferenceServerClient(AbstractEndpoint endpoint, HttpConfig httpConfig) {
    this.endpoint = endpoint;
    this.config = httpConfig;
    if (!httpConfig.isKeepAlive()) {
      // the JDK client pools connections; this property turns reuse off process-wide
      System.setProperty("jdk.httpclient.keepalive.timeout", "0");
    }
    System.setProperty("jdk.httpclient.connectionPoolSize", Integer.toString(httpConfig.getMaxConnectionCount()));
    this.executor = Executors.newFixedThreadPool(httpConfig.getIoThreadNum(), r -> {
      Thread t = new Thread(r, "triton-client-io");
      t.setDaemon(true);
      return t;
    });
    this.http = HttpClient.newBuilder()
                    .version(HttpClient.Version.HTTP_1_1)
                    .connectTimeout(Duration.ofMillis(httpConfig.getConnectTimeout()))
                    .executor(executor)
                    .build();
  }

  /** Attempts per request on I/O errors (>= 1; endpoint rotation happens between attempts). */
  public void setRetryCnt(int retryCnt) {
    Util.checkArgument(retryCnt > 0, "retryCnt must be > 0");
    this.retryCnt = retryCnt;
  }

  public int getRetryCnt() { return retryCnt; }

  // ------------------------------------------------------------ control plane
  public boolean isServerLive() throws InferenceException { return get("/v2/health/live").statusCode() == 200; }

  public boolean isServerReady() throws InferenceException { return get("/v2/health/ready").statusCode() == 200; }

  public boolean isModelReady(String model, String version) throws InferenceException {
    return get(modelPath(model, version) + "/ready").statusCode() == 200;
  }

  public Map<String, Object> getServerMetadata() throws InferenceException { return getJson("/v2"); }

  public Map<String, Object> getModelMetadata(String model, String version) throws InferenceException {
    return getJson(modelPath(model, version));
  }

  public Map<String, Object> getModelConfig(String model, String version) throws InferenceException {
    return getJson(modelPath(model, version) + "/config");
  }

  private static String enc(String s) { return URLEncoder.encode(s, StandardCharsets.UTF_8).replace("+", "%20"); }

  private static String modelPath(String model, String version) {
    String p = "/v2/models/" + enc(model);
    if (!Util.isEmpty(version)) p += "/versions/" + enc(version);
    return p;
  }

  private HttpResponse<byte[]> get(String path) throws InferenceException {
    return send(path, null, null, new LinkedHashMap<>());
  }

  private Map<String, Object> getJson(String path) throws InferenceException {
    HttpResponse<byte[]> r = get(path);
    String body = new String(r.body(), StandardCharsets.UTF_8);
    if (r.statusCode() != 200) throw error(r.statusCode(), body);
    return Json.parseObject(body);
  }

  private static InferenceException error(int status, String body) {
    String msg = body;
    try {
      Object e = Json.parseObject(body).get("error");
      if (e != null) msg = e.toString();
    } catch (RuntimeException ignored) {
      // not JSON: keep the raw body
    }
    if (status == 499) msg = "Deadline Exceeded";
    return new InferenceException(msg, status);
  }

  private HttpResponse<byte[]> send(String path, byte[] body, Integer headerLen, Map<String, String> headers)
      throws InferenceException {
    Exception last = null;
    int attempts = Math.max(1, retryCnt);
    for (int i = 0; i < attempts; i++) {
      try {
        HttpRequest req = buildRequest(endpoint.getEndpoint(), path, body, headerLen, headers);
        return http.send(req, HttpResponse.BodyHandlers.ofByteArray());
      } catch (IOException e) {
        last = e;  // connection-level failure: retry (possibly on another endpoint)
      } catch (InterruptedException e) {
        Thread.currentThread().interrupt();
        throw new InferenceException(e);
      } catch (Exception e) {
        throw new InferenceException(e);
      }
    }
    throw new InferenceException(last);
  }

  private HttpRequest buildRequest(String ep, String path, byte[] body, Integer headerLen, Map<String, String> headers) {
    HttpRequest.Builder b = HttpRequest.newBuilder(URI.create("http://" + ep + path))
                                .timeout(Duration.ofMillis(config.getReadTimeout()));
    for (Map.Entry<String, String> h : headers.entrySet()) b.header(h.getKey(), h.getValue());
    if (body == null) return b.GET().build();
    if (headerLen != null) {
      b.header(HEADER_LEN, headerLen.toString());
      b.header("Content-Type", "application/octet-stream");
    } else {
      b.header("Content-Type", "application/json");
    }
    return b.POST(HttpRequest.BodyPublishers.ofByteArray(body)).build();
  }

  // --------------------------------------------------------------- inference
  /** Inference arguments (reference InferArguments, :377-468). */
  public static class InferArguments {
    private final String modelName;
    private final List<InferInput> inputs;
    private List<InferRequestedOutput> outputs;
    private String modelVersion;
    private String requestId;
    private long sequenceId;
    private String sequenceIdStr;
    private boolean sequenceStart;
    private boolean sequenceEnd;
    private long priority;
    private int timeout;
    private final Map<String, String> headers = new LinkedHashMap<>();
    private final Map<String, String> queryParams = new LinkedHashMap<>();
    private final Parameters custom = new Parameters();

    public InferArguments(String modelName, List<InferInput> inputs, List<InferRequestedOutput> outputs) {
      Util.checkArgument(!Util.isEmpty(modelName), "model name must not be empty");
      Util.checkArgument(!Util.isEmpty(inputs), "inputs must not be empty");
      this.modelName = modelName;
      this.inputs = inputs;
      this.outputs = outputs;
    }

    public InferArguments(String modelName, List<InferInput> inputs) { this(modelName, inputs, null); }

    public InferArguments(String modelName, InferInput... inputs) { this(modelName, Arrays.asList(inputs), null); }

    public InferArguments setOutputs(List<InferRequestedOutput> outputs) {
      this.outputs = outputs;
      return this;
    }

    public InferArguments setModelVersion(String modelVersion) {
      this.modelVersion = modelVersion;
      return this;
    }

    public InferArguments setRequestId(String requestId) {
      this.requestId = requestId;
      return this;
    }

    public InferArguments setSequenceId(long sequenceId) {
      this.sequenceId = sequenceId;
      this.sequenceIdStr = null;
      return this;
    }

    /** String correlation id (Triton's string sequence-id form). */
    public InferArguments setSequenceId(String sequenceId) {
      this.sequenceIdStr = sequenceId;
      this.sequenceId = 0;
      return this;
    }

    public InferArguments setSequenceStart(boolean sequenceStart) {
      this.sequenceStart = sequenceStart;
      return this;
    }

    public InferArguments setSequenceEnd(boolean sequenceEnd) {
      this.sequenceEnd = sequenceEnd;
      return this;
    }

    public InferArguments setPriority(long priority) {
      this.priority = priority;
      return this;
    }

    /** Server-side timeout in microseconds. */
    public InferArguments setTimeout(int timeout) {
      this.timeout = timeout;
      return this;
    }

    public InferArguments setHeader(String key, String value) {
      headers.put(key, value);
      return this;
    }

    public InferArguments addQueryParam(String key, String value) {
      queryParams.put(key, value);
      return this;
    }

    /** Custom request parameter (bool / integer / float / string). */
    public InferArguments setParameter(String key, Object value) {
      custom.put(key, value);
      return this;
    }
  }

  /** JSON header + concatenated binary inputs; returns {body, headerLength or null}. */
  static Object[] buildInferBody(InferArguments a) {
    Map<String, Object> req = new LinkedHashMap<>();
    if (!Util.isEmpty(a.requestId)) req.put("id", a.requestId);
    Map<String, Object> params = new LinkedHashMap<>(a.custom.asMap());
    if (a.sequenceIdStr != null) {
      params.put("sequence_id", a.sequenceIdStr);
    } else if (a.sequenceId != 0) {
      params.put("sequence_id", new Json.Unsigned(a.sequenceId));
    }
    if (a.sequenceIdStr != null || a.sequenceId != 0) {
      params.put("sequence_start", a.sequenceStart);
      params.put("sequence_end", a.sequenceEnd);
    }
    if (a.priority != 0) params.put("priority", new Json.Unsigned(a.priority));
    if (a.timeout != 0) params.put("timeout", (long) a.timeout);
    if (Util.isEmpty(a.outputs)) params.put("binary_data_output", true);
    if (!params.isEmpty()) req.put("parameters", params);
    List<Object> ins = new ArrayList<>();
    boolean anyBinary = false;
    for (InferInput in : a.inputs) {
      ins.add(in.getTensor().toJson());
      anyBinary |= in.isBinary();
    }
    req.put("inputs", ins);
    if (!Util.isEmpty(a.outputs)) {
      List<Object> outs = new ArrayList<>();
      for (InferRequestedOutput o : a.outputs) outs.add(o.getTensor().toJson());
      req.put("outputs", outs);
    }
    byte[] header = Json.writeBytes(req);
    if (!anyBinary) return new Object[] {header, null};
    ByteArrayOutputStream body = new ByteArrayOutputStream(header.length + 4096);
    body.write(header, 0, header.length);
    for (InferInput in : a.inputs) {
      if (in.isBinary()) body.write(in.getBinaryData(), 0, in.getBinaryData().length);
    }
    return new Object[] {body.toByteArray(), header.length};
  }

  private static String inferPath(InferArguments a) {
    StringBuilder p = new StringBuilder(modelPath(a.modelName, a.modelVersion)).append("/infer");
    char sep = '?';
    for (Map.Entry<String, String> q : a.queryParams.entrySet()) {
      p.append(sep).append(enc(q.getKey())).append('=').append(enc(q.getValue()));
      sep = '&';
    }
    return p.toString();
  }

  private static InferResult toResult(HttpResponse<byte[]> r) throws InferenceException {
    if (r.statusCode() != 200) throw error(r.statusCode(), new String(r.body(), StandardCharsets.UTF_8));
    int hl = r.headers().firstValue(HEADER_LEN).map(Integer::parseInt).orElse(-1);
    return new InferResult(r.body(), hl);
  }

  /** Synchronous inference (reference :252-366). */
  public InferResult infer(InferArguments arg) throws InferenceException {
    Object[] b = buildInferBody(arg);
    return toResult(send(inferPath(arg), (byte[]) b[0], (Integer) b[1], arg.headers));
  }

  public InferResult infer(String modelName, List<InferInput> inputs, List<InferRequestedOutput> outputs)
      throws InferenceException {
    return infer(new InferArguments(modelName, inputs, outputs));
  }

  /** Non-blocking inference on the client's I/O pool (not in the reference Java subset). */
  public CompletableFuture<InferResult> inferAsync(InferArguments arg) {
    final HttpRequest req;
    try {
      Object[] b = buildInferBody(arg);
      req = buildRequest(endpoint.getEndpoint(), inferPath(arg), (byte[]) b[0], (Integer) b[1], arg.headers);
    } catch (Exception e) {
      CompletableFuture<InferResult> f = new CompletableFuture<>();
      f.completeExceptionally(e instanceof InferenceException ? e : new InferenceException(e));
      return f;
    }
    return http.sendAsync(req, HttpResponse.BodyHandlers.ofByteArray()).thenApply(r -> {
      try {
        return toResult(r);
      } catch (InferenceException e) {
        throw new CompletionException(e);
      }
    });
  }

  @Override public void close() { executor.shutdownNow(); }

  /** For logs: the JSON text of a request header (no binary tail). */
  public static String describe(InferArguments a) {
    Object[] b = buildInferBody(a);
    byte[] body = (byte[]) b[0];
    int n = b[1] == null ? body.length : (Integer) b[1];
    return new String(body, 0, n, StandardCharsets.UTF_8);
  }

  /** The tensor list of a request, for inspection. */
  public static List<IOTensor> tensors(InferArguments a) {
    List<IOTensor> out = new ArrayList<>();
    for (InferInput in : a.inputs) out.add(in.getTensor());
    return out;
  }
}
