package triton.client;

import java.util.ArrayList;
import java.util.List;

import triton.client.pojo.DataType;
import triton.client.pojo.IOTensor;
import triton.client.pojo.Parameters;

/**
 * One input tensor of an inference request (reference InferInput.java:52-353).
 * {@code setData(array, isBinary)} either encodes the values little-endian
 * for the binary-data extension or keeps them for the JSON "data" field.
 */
public class InferInput {
  private final String name;
  private final long[] shape;
  private final DataType dataType;
  private final Parameters parameters = new Parameters();
  private byte[] binaryData;
  private List<Object> jsonData;

  public InferInput(String name, long[] shape, DataType dataType) {
    Util.checkArgument(!Util.isEmpty(name), "input name must not be empty");
    this.name = name;
    this.shape = shape.clone();
    this.dataType = dataType;
  }

  public String getName() { return name; }

  public long[] getShape() { return shape.clone(); }

  public DataType getDataType() { return dataType; }

  public Parameters getParameters() { return parameters; }

  /** Encoded tensor bytes when the input is sent as binary, else null. */
  public byte[] getBinaryData() { return binaryData; }

  public boolean isBinary() { return binaryData != null; }

  private void checkCount(int n) {
    long want = Util.elemNumFromShape(shape);
    Util.checkArgument(n == want, "input %s: %d values for shape of %d elements", name, n, want);
  }

  private void setBinary(byte[] b) {
    binaryData = b;
    jsonData = null;
    parameters.put(Parameters.KEY_BINARY_DATA_SIZE, (long) b.length);
  }

  private void setJson(List<Object> d) {
    Util.checkArgument(dataType != DataType.FP16 && dataType != DataType.BF16,
        "input %s: %s can only be sent as binary data", name, dataType);
    jsonData = d;
    binaryData = null;
    parameters.remove(Parameters.KEY_BINARY_DATA_SIZE);
  }

  public void setData(boolean[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (boolean v : data) d.add(v);
      setJson(d);
    }
  }

  public void setData(byte[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (byte v : data) d.add(dataType.signed ? (long) v : (long) (v & 0xff));
      setJson(d);
    }
  }

  public void setData(short[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (short v : data) d.add(dataType.signed ? (long) v : (long) (v & 0xffff));
      setJson(d);
    }
  }

  public void setData(int[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (int v : data) d.add(dataType.signed ? (long) v : (v & 0xffffffffL));
      setJson(d);
    }
  }

  public void setData(long[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (long v : data) d.add(dataType == DataType.UINT64 ? new triton.client.pojo.Json.Unsigned(v) : (Object) v);
      setJson(d);
    }
  }

  public void setData(float[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (float v : data) d.add(v);
      setJson(d);
    }
  }

  public void setData(double[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(dataType, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (double v : data) d.add(v);
      setJson(d);
    }
  }

  public void setData(String[] data, boolean isBinaryData) {
    checkCount(data.length);
    if (isBinaryData) {
      setBinary(BinaryProtocol.toBytes(DataType.BYTES, data));
    } else {
      List<Object> d = new ArrayList<>(data.length);
      for (String v : data) d.add(v);
      setJson(d);
    }
  }

  /** The "inputs" entry of the request header. */
  public IOTensor getTensor() {
    Util.checkArgument(binaryData != null || jsonData != null, "input %s has no data", name);
    IOTensor t = new IOTensor();
    t.setName(name);
    t.setShape(shape);
    t.setDatatype(dataType);
    if (!parameters.isEmpty()) t.setParameters(parameters);
    if (jsonData != null) t.setData(jsonData);
    return t;
  }
}
