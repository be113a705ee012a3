package triton.client;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import triton.client.pojo.DataType;
import triton.client.pojo.IOTensor;
import triton.client.pojo.InferenceResponse;
import triton.client.pojo.Json;
import triton.client.pojo.Parameters;

/**
 * Parsed inference response (reference InferResult.java:58-318): the JSON
 * header (its length from {@code Inference-Header-Content-Length}, or the
 * whole body when absent) followed by the binary outputs in header order.
 * Getters convert from either the binary slice or the JSON "data" list.
 */
public class InferResult {
  /** Byte range of one binary output inside the body. */
  public static class Index {
    public final int start;
    public final int length;

    public Index(int start, int length) {
      this.start = start;
      this.length = length;
    }
  }

  private final InferenceResponse response;
  private final Map<String, Index> nameToBinaryIdx = new HashMap<>();
  private final byte[] body;

  /**
   * @param body raw HTTP response body
   * @param headerLength value of Inference-Header-Content-Length, or -1 when the body is all JSON
   */
  public InferResult(byte[] body, int headerLength) throws InferenceException {
    this.body = body;
    int jsonLen = headerLength < 0 ? body.length : headerLength;
    if (jsonLen > body.length) throw new InferenceException("header length " + jsonLen + " exceeds body " + body.length);
    String json = new String(body, 0, jsonLen, StandardCharsets.UTF_8);
    try {
      response = InferenceResponse.fromJson(Json.parseObject(json));
    } catch (IllegalArgumentException e) {
      throw new InferenceException("malformed response header: " + e.getMessage());
    }
    int pos = jsonLen;
    for (IOTensor t : response.getOutputs()) {
      Parameters p = t.getParameters();
      Long size = p == null ? null : p.getLong(Parameters.KEY_BINARY_DATA_SIZE);
      if (size == null) continue;
      if (pos + size > body.length) throw new InferenceException("output " + t.getName() + " overruns the body");
      nameToBinaryIdx.put(t.getName(), new Index(pos, size.intValue()));
      pos += size.intValue();
    }
  }

  public InferenceResponse getResponse() { return response; }

  public Map<String, Index> getNameToBinaryIdx() { return nameToBinaryIdx; }

  public byte[] getBinaryData() { return body; }

  public String getModelName() { return response.getModelName(); }

  public String getModelVersion() { return response.getModelVersion(); }

  public String getId() { return response.getId(); }

  public List<String> getOutputs() {
    List<String> names = new ArrayList<>();
    for (IOTensor t : response.getOutputs()) names.add(t.getName());
    return names;
  }

  public long[] getShape(String output) { return tensor(output).getShape(); }

  public DataType getDatatype(String output) { return tensor(output).getDatatype(); }

  private IOTensor tensor(String output) {
    IOTensor t = response.getOutputByName(output);
    if (t == null) throw new IllegalArgumentException("no output named " + output);
    return t;
  }

  private ByteBuffer binary(String output) {
    Index idx = nameToBinaryIdx.get(output);
    if (idx == null) return null;
    return ByteBuffer.wrap(body, idx.start, idx.length).slice().order(ByteOrder.LITTLE_ENDIAN);
  }

  private int count(IOTensor t, ByteBuffer b) {
    if (b == null) return t.getData() == null ? 0 : t.getData().size();
    return b.remaining() / Math.max(1, t.getDatatype().numByte);
  }

  /** Element i of an output as a double (binary or JSON). */
  private double num(IOTensor t, ByteBuffer b, int i) {
    if (b == null) {
      Object o = t.getData().get(i);
      if (o instanceof Boolean) return ((Boolean) o) ? 1 : 0;
      return ((Number) o).doubleValue();
    }
    DataType dt = t.getDatatype();
    int off = i * dt.numByte;
    switch (dt) {
      case BOOL: return b.get(off) != 0 ? 1 : 0;
      case INT8: return b.get(off);
      case UINT8: return b.get(off) & 0xff;
      case INT16: return b.getShort(off);
      case UINT16: return b.getShort(off) & 0xffff;
      case INT32: return b.getInt(off);
      case UINT32: return b.getInt(off) & 0xffffffffL;
      case INT64: return b.getLong(off);
      case UINT64: return new Json.Unsigned(b.getLong(off)).doubleValue();
      case FP16: return BinaryProtocol.halfToFloat(b.getShort(off));
      case BF16: return BinaryProtocol.bf16ToFloat(b.getShort(off));
      case FP32: return b.getFloat(off);
      case FP64: return b.getDouble(off);
      default: throw new IllegalArgumentException(dt + " is not numeric");
    }
  }

  /** Element i as a long, exact for 64-bit integers. */
  private long lng(IOTensor t, ByteBuffer b, int i) {
    if (b == null) {
      Object o = t.getData().get(i);
      if (o instanceof Boolean) return ((Boolean) o) ? 1 : 0;
      return ((Number) o).longValue();
    }
    DataType dt = t.getDatatype();
    if (dt == DataType.INT64 || dt == DataType.UINT64) return b.getLong(i * 8);
    return (long) num(t, b, i);
  }

  public boolean[] getOutputAsBool(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    boolean[] r = new boolean[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = num(t, b, i) != 0;
    return r;
  }

  public byte[] getOutputAsByte(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    byte[] r = new byte[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = (byte) lng(t, b, i);
    return r;
  }

  public short[] getOutputAsShort(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    short[] r = new short[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = (short) lng(t, b, i);
    return r;
  }

  public int[] getOutputAsInt(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    int[] r = new int[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = (int) lng(t, b, i);
    return r;
  }

  public long[] getOutputAsLong(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    long[] r = new long[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = lng(t, b, i);
    return r;
  }

  public float[] getOutputAsFloat(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    float[] r = new float[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = (float) num(t, b, i);
    return r;
  }

  public double[] getOutputAsDouble(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    double[] r = new double[count(t, b)];
    for (int i = 0; i < r.length; i++) r[i] = num(t, b, i);
    return r;
  }

  /** BYTES output (binary length-prefixed elements or JSON strings), also classification results. */
  public String[] getOutputAsString(String output) {
    IOTensor t = tensor(output);
    ByteBuffer b = binary(output);
    List<String> r = new ArrayList<>();
    if (b == null) {
      if (t.getData() != null) {
        for (Object o : t.getData()) r.add(String.valueOf(o));
      }
    } else {
      while (b.remaining() >= 4) {
        int len = b.getInt();
        byte[] s = new byte[len];
        b.get(s);
        r.add(new String(s, StandardCharsets.UTF_8));
      }
    }
    return r.toArray(new String[0]);
  }
}
