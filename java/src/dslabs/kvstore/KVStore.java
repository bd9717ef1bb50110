package dslabs.kvstore;

import dslabs.framework.Application;
import dslabs.framework.Command;
import dslabs.framework.Result;
import java.util.HashMap;
import java.util.Map;
import java.util.Objects;
import lombok.EqualsAndHashCode;
import lombok.ToString;

/**
 * The lab1 key-value store (DESIGN.md §11): Get -> GetResult(value) or KeyNotFound, Put -> PutOk,
 * Append -> AppendResult(new value), as KVStoreWorkload expects (KVStoreWorkload.java:40-66). The
 * commands and results are the reference's (labs/lab1-clientserver/src/dslabs/kvstore/KVStore.java),
 * written as records with the same accessors, equality and (Lombok-format) toString -- PaxosTest's
 * hasCommand predicate names carry it. On the device a key is a key id (<= 3
 * keys) and a value a sequence of <= 9 equal-length workload tokens (amokv.hpp).
 */
@ToString
@EqualsAndHashCode
public class KVStore implements Application {

  public interface KVStoreCommand extends Command {}

  public interface SingleKeyCommand extends KVStoreCommand {
    String key();
  }

  public record Get(String key) implements SingleKeyCommand {
    public Get {
      Objects.requireNonNull(key);
    }

    @Override
    public String toString() {
      return "KVStore.Get(key=" + key + ")";
    }

    @Override
    public boolean readOnly() {
      return true;
    }
  }

  public record Put(String key, String value) implements SingleKeyCommand {
    public Put {
      Objects.requireNonNull(key);
      Objects.requireNonNull(value);
    }

    @Override
    public String toString() {
      return "KVStore.Put(key=" + key + ", value=" + value + ")";
    }
  }

  public record Append(String key, String value) implements SingleKeyCommand {
    public Append {
      Objects.requireNonNull(key);
      Objects.requireNonNull(value);
    }

    @Override
    public String toString() {
      return "KVStore.Append(key=" + key + ", value=" + value + ")";
    }
  }

  public interface KVStoreResult extends Result {}

  public record GetResult(String value) implements KVStoreResult {
    public GetResult {
      Objects.requireNonNull(value);
    }

    @Override
    public String toString() {
      return "KVStore.GetResult(value=" + value + ")";
    }
  }

  public record KeyNotFound() implements KVStoreResult {
    @Override
    public String toString() {
      return "KVStore.KeyNotFound()";
    }
  }

  public record PutOk() implements KVStoreResult {
    @Override
    public String toString() {
      return "KVStore.PutOk()";
    }
  }

  public record AppendResult(String value) implements KVStoreResult {
    public AppendResult {
      Objects.requireNonNull(value);
    }

    @Override
    public String toString() {
      return "KVStore.AppendResult(value=" + value + ")";
    }
  }

  private final Map<String, String> data = new HashMap<>();

  @Override
  public KVStoreResult execute(Command command) {
    if (command instanceof Get g) {
      String v = data.get(g.key());
      return v == null ? new KeyNotFound() : new GetResult(v);
    }
    if (command instanceof Put p) {
      data.put(p.key(), p.value());
      return new PutOk();
    }
    if (command instanceof Append a) {
      String v = data.getOrDefault(a.key(), "") + a.value();
      data.put(a.key(), v);
      return new AppendResult(v);
    }
    throw new IllegalArgumentException();
  }
}
