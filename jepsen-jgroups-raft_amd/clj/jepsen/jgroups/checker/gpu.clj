(ns jepsen.jgroups.checker.gpu
  "Drop-in for (checker/linearizable {:model m :algorithm :linear}) backed by
  liblincheck.so (include/lincheck.h) through JNA. Reference call sites replaced:
  src/jepsen/jgroups/workload/register.clj:109-111 and counter.clj:135-137 (SURVEY
  numbering; file lines :250-254). Not executable in the build container (no JVM):
  the Python ctypes harness (lincheck/_lib.py) makes the same calls with the same
  arrays and is what the tests exercise."
  (:require [jepsen.checker :as checker]
            [jepsen.independent :as independent]
            [knossos.model :as model])
  (:import (com.sun.jna Native NativeLibrary Function Memory)
           (knossos.model CASRegister)))

(def ^:private lib (delay (NativeLibrary/getInstance "lincheck")))

(defn- f [name] (.getFunction ^NativeLibrary @lib name))

(def type-code {:invoke 0 :ok 1 :fail 2 :info 3})
(def f-code {:read 0 :write 1 :cas 2 :add 3 :decr 4 :add-and-get 5 :decr-and-get 6})

(defn- encode
  "Histories (seq of op vectors) -> SoA primitive arrays in lincheck.h order."
  [histories]
  (let [ops   (vec (apply concat histories))
        n     (count ops)
        off   (long-array (reductions + 0 (map count histories)))
        index (long-array n) process (int-array n) type (byte-array n) fs (byte-array n)
        v0 (long-array n) v1 (long-array n) vflags (byte-array n)]
    (dotimes [i n]
      (let [op (nth ops i) v (:value op)]
        (aset index i (long (:index op i)))
        (aset process i (int (:process op)))
        (aset type i (byte (type-code (:type op))))
        (aset fs i (byte (f-code (:f op))))
        (cond (nil? v)    (aset vflags i (byte 0))
              (vector? v) (do (aset vflags i (byte 2)) (aset v0 i (long (v 0))) (aset v1 i (long (v 1))))
              :else       (do (aset vflags i (byte 1)) (aset v0 i (long v))))))
    {:off off :index index :process process :type type :f fs :v0 v0 :v1 v1 :vflags vflags}))

(defn check-histories
  "One lc_check call for many histories; returns a vector of Knossos-keyed maps."
  [model-kind init histories opts]
  (let [{:keys [off index process type f v0 v1 vflags]} (encode histories)
        k (count histories)
        valid (byte-array k) fail (long-array k) finv (long-array k) prev (long-array k)
        explored (long-array k) errs (int-array k) err (byte-array 512)
        rc (.invokeInt ^Function (f "lc_check")
                       (object-array [(int model-kind) (long init) (int k) off index process type
                                      f v0 v1 vflags (int (:gpus opts 0)) (long (:max-configs opts 0))
                                      (int 0) valid fail finv prev explored errs err (int 512)]))]
    (when-not (zero? rc)
      (throw (ex-info (String. err 0 (int (or (first (keep-indexed #(when (zero? %2) %1) err)) 512)))
                      {:rc rc})))
    (vec (for [i (range k)]
           (let [ops (nth histories i)
                 at  (fn [idx] (first (filter #(= idx (:index %)) ops)))]
             (cond-> {:valid?   (case (aget valid i) 1 true 0 false :unknown)
                      :analyzer :linear
                      :explored (aget explored i)}
               (zero? (aget valid i)) (assoc :op (at (aget fail i))
                                             :previous-ok (at (aget prev i))
                                             :last-op (at (aget prev i)))))))))

(defn- model-kind [m]
  (cond (instance? CASRegister m) [1 0]
        (= "CounterModel" (.getSimpleName (class m))) [2 (long (:value m))]
        :else nil))

(defn linearizable
  "Same options as checker/linearizable. Models the GPU does not implement (e.g. the
  election workload's LeaderModel, leader.clj:63-75) fall back to Knossos."
  [{:keys [model] :as opts}]
  (if-let [[kind init] (model-kind model)]
    (reify checker/Checker
      (check [_ test history copts]
        (first (check-histories kind init [(filterv #(integer? (:process %)) history)] opts))))
    (checker/linearizable opts)))
