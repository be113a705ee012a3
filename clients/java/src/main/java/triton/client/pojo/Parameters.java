package triton.client.pojo;

import java.util.LinkedHashMap;
import java.util.Map;

/**
 * A "parameters" object: string keys to bool / integer / float / string
 * values, with typed getters that accept any JSON numeric representation
 * (reference pojo/Parameters.java:55-236).
 */
public class Parameters {
  public static final String KEY_BINARY_DATA_SIZE = "binary_data_size";
  public static final String KEY_BINARY_DATA = "binary_data";
  public static final String KEY_CLASSIFICATION = "classification";

  private final Map<String, Object> params;

  public Parameters() { this.params = new LinkedHashMap<>(); }

  public Parameters(Map<String, Object> params) {
    this.params = params == null ? new LinkedHashMap<>() : new LinkedHashMap<>(params);
  }

  public Object put(String key, Object value) { return params.put(key, value); }

  /** Stores an unsigned 64-bit value (serialised without sign). */
  public Object putUnsignedLong(String key, long value) {
    return params.put(key, new Json.Unsigned(value));
  }

  public Object remove(String key) { return params.remove(key); }

  public boolean isEmpty() { return params.isEmpty(); }

  public Object get(String key) { return params.get(key); }

  public Map<String, Object> asMap() { return params; }

  public Boolean getBool(String name) {
    Object v = params.get(name);
    if (v == null) return null;
    if (v instanceof Boolean) return (Boolean) v;
    if (v instanceof Number) return ((Number) v).longValue() != 0;
    return Boolean.parseBoolean(v.toString());
  }

  public Integer getInt(String name) {
    Object v = params.get(name);
    if (v == null) return null;
    if (v instanceof Number) return ((Number) v).intValue();
    return Integer.parseInt(v.toString());
  }

  public Long getLong(String name) {
    Object v = params.get(name);
    if (v == null) return null;
    if (v instanceof Number) return ((Number) v).longValue();
    return Long.parseLong(v.toString());
  }

  public Float getFloat(String name) {
    Object v = params.get(name);
    if (v == null) return null;
    if (v instanceof Number) return ((Number) v).floatValue();
    return Float.parseFloat(v.toString());
  }

  public Double getDouble(String name) {
    Object v = params.get(name);
    if (v == null) return null;
    if (v instanceof Number) return ((Number) v).doubleValue();
    return Double.parseDouble(v.toString());
  }

  public String getString(String name) {
    Object v = params.get(name);
    return v == null ? null : v.toString();
  }
}
